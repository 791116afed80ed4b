// ba_kernel.hip — sliding-window bundle adjustment on MI355X (gfx950), one workgroup per window.
//
// Replaces ceres::Solve(SPARSE_SCHUR/DENSE_SCHUR, LEVENBERG_MARQUARDT) as driven by
// Optimizer::RunLocalBA / RunBA / RunVIBA / SolvePnP (src/optimization/Optimizer.cpp:83-966):
//   * residual/Jacobian of BAFactor / PnPFactor (src/optimization/Factors.cpp:33-612) per
//     observation lane, HuberLoss + Corrector scaling (ceres loss_function.cc:48-62,
//     corrector.cc:42-156), InertialFactorFixedGravity (Factors.cpp:1299-1485) per factor lane;
//   * Ceres-2.0 trust-region LM control flow (trust_region_minimizer.cc:67-826,
//     levenberg_marquardt_strategy.cc:66-160) kept ON DEVICE in LDS, so a whole solve is one
//     launch with no host round trip;
//   * Jacobi column scaling, LM diagonal, Schur complement over the points
//     (schur_eliminator_impl.h:179-377) with the pose-pose block as an LDS-staged GEMM,
//     right-looking Cholesky of the reduced system in LDS, back-substitution.
// All reductions are fixed-order (wave shuffles + ordered wave combine): results are bitwise
// reproducible run to run (no floating-point atomics).
#include <float.h>
#include <hip/hip_runtime.h>

#include "ba_types.h"
#include "ba_factor_dev.h"
#include "lie_dev.h"

namespace vio360 {

constexpr int VI_KMAX = 10;  // VIBA windows on this path: K <= 10 (ni = 3K+6 <= 36)
constexpr int NI_MAX = 3 * VI_KMAX + 6;

struct LmState {
    double radius, decrease_factor;
    double x_cost, cand_cost, min_cost, model_change, x_norm, gmax;
    double initial_cost, final_cost, fixed_cost, iter_cost, step_eval_current;
    double step_norm, cand_x_norm2, rel;
    int iteration, nsucc, nunsucc, consecutive_invalid;
    int termination, done, step_ok, valid, fail, need_jac, pnp_round;
};

struct __align__(16) BaShared {
    double S[BA_NF_MAX * (BA_NF_MAX + 1)];  // row stride s_ld(nf) (odd), rows padded to 16-row tiles
    double stage[BA_STAGE];      // with S: the Schur panels At | Bt (k-major, see schur_gemm)
    double gcol[BA_GCOL];
    double b[BA_NF_MAX], s_f[BA_NF_MAX], g_f[BA_NF_MAX], colsq_f[BA_NF_MAX], D_f[BA_NF_MAX];
    double U[BA_KMAX][27];
    double pc[BA_KMAX][36];      // Rwb(9) twb(3) Rbw(9) tbw(3) Rcw(9) tcw(3) at the point being evaluated
    double pinit[BA_KMAX][24];   // projected R_init(9) t_init(3) R_cb(9) t_cb(3)
    double Rcb_raw[BA_KMAX][9];
    double imu_r[VI_KMAX][9];
    double imu_J[VI_KMAX][108];  // per factor 9x12: [vi | bg | ba | vj]
    double red[BA_THREADS / 64 + 4];
    double redm[BA_THREADS / 64 + 4];
    LmState st;
    unsigned long long prof_acc[16];
    unsigned long long prof_last;
    int prof_on;
    int chol_bad;
    int posef[BA_KMAX];          // copy of BaWin::pose_f (per-lane indexed in the Schur fill)
};
static_assert(sizeof(BaShared) <= 160 * 1024, "BaShared exceeds the 160 KB LDS of a gfx950 CU");
static_assert(offsetof(BaShared, stage) == offsetof(BaShared, S) + sizeof(double) * BA_NF_MAX * (BA_NF_MAX + 1),
              "Schur panels span S and stage contiguously");

// row stride of S: tile-padded size, odd (conflict-free column walks)
__host__ __device__ constexpr int s_ld(int nf) { return (16 * ((nf + 15) >> 4)) | 1; }
static_assert(16 * ((BA_NF_MAX + 15) >> 4) * s_ld(BA_NF_MAX) <= BA_NF_MAX * (BA_NF_MAX + 1), "S padding");

// per-phase shader-clock accounting (diagnostic; enabled when BaPools::prof != nullptr)
enum { PF_SETUP = 0, PF_EVAL_J, PF_LIN, PF_PREP, PF_GEMM, PF_CHOL, PF_BACKSUB, PF_CAND, PF_EVAL_C, PF_CTRL, PF_POST, PF_FILL };
__device__ __forceinline__ void prof_mark(BaShared& sh, int slot) {
    if (sh.prof_on && threadIdx.x == 0) {
        unsigned long long t = __builtin_amdgcn_s_memtime();
        sh.prof_acc[slot] += t - sh.prof_last;
        sh.prof_last = t;
    }
}

// ------------------------------------------------------------------------------------------
// fixed-order block reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_down(v, off, 64));
    return v;
}
__device__ __forceinline__ double block_sum(double v, double* red) {
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = 0.0;
#pragma unroll
    for (int w = 0; w < BA_THREADS / 64; ++w) r += red[w];
    return r;
}
__device__ __forceinline__ double block_max(double v, double* red) {
    v = wave_max(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = 0.0;
#pragma unroll
    for (int w = 0; w < BA_THREADS / 64; ++w) r = fmax(r, red[w]);
    return r;
}

// ------------------------------------------------------------------------------------------
// InertialFactorFixedGravity::Evaluate (Factors.cpp:1326-1485); pose Jacobians are identically
// zero in the reference, so only [vi | bg | ba | vj] columns are produced (9x12).
__device__ inline void imu_log(const double* R, double* w) {  // Factors.cpp:1507-1519
    double c = fmax(-1.0, fmin(1.0, (R[0] + R[4] + R[8] - 1.0) / 2.0));
    double th = acos(c);
    double v[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};
    double f = th < 1e-6 ? 0.5 : th / (2.0 * sin(th));
    w[0] = f * v[0]; w[1] = f * v[1]; w[2] = f * v[2];
}
__device__ __noinline__ void imu_eval(const vio_preint& p, const double* sqi, const double* g, const double* pci,
                                const double* pcj, const double* vi, const double* bg, const double* ba,
                                const double* vj, bool want_jac, double* r, double* J) {
    const double* Rwi = pci;
    const double* twi = pci + 3 * 3;
    const double* Rwj = pcj;
    const double* twj = pcj + 9;
    const double* Rbwi = pci + 12;  // R_wbi^T
    double dt = p.dt_total;
    double DR[9], DV[3], DP[3], JRg[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) { DR[i] = (double)p.delta_R[i]; JRg[i] = (double)p.J_Rg[i]; }
#pragma unroll
    for (int i = 0; i < 3; ++i) { DV[i] = (double)p.delta_V[i]; DP[i] = (double)p.delta_P[i]; }
    double dbg[3], dba[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) { dbg[i] = bg[i] - (double)p.gyro_bias[i]; dba[i] = ba[i] - (double)p.accel_bias[i]; }
    if (nrm3(dbg) > 1e-6 || nrm3(dba) > 1e-6) {
        double w[3], E[9], M[9];
        m3vec(JRg, dbg, w);
        so3_exp(w, E);
        m3mul(DR, E, M);
#pragma unroll
        for (int i = 0; i < 9; ++i) DR[i] = M[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            DV[i] += (double)p.J_Vg[3 * i] * dbg[0] + (double)p.J_Vg[3 * i + 1] * dbg[1] + (double)p.J_Vg[3 * i + 2] * dbg[2]
                   + (double)p.J_Va[3 * i] * dba[0] + (double)p.J_Va[3 * i + 1] * dba[1] + (double)p.J_Va[3 * i + 2] * dba[2];
            DP[i] += (double)p.J_Pg[3 * i] * dbg[0] + (double)p.J_Pg[3 * i + 1] * dbg[1] + (double)p.J_Pg[3 * i + 2] * dbg[2]
                   + (double)p.J_Pa[3 * i] * dba[0] + (double)p.J_Pa[3 * i + 1] * dba[1] + (double)p.J_Pa[3 * i + 2] * dba[2];
        }
    }
    double raw[9];
    {
        double A[9], B[9];
        m3tmul(DR, Rbwi, A);  // DR^T * R_bwi
        m3mul(A, Rwj, B);
        imu_log(B, raw);
        double tv[3], ev[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) tv[i] = vj[i] - vi[i] - g[i] * dt;
        m3vec(Rbwi, tv, ev);
#pragma unroll
        for (int i = 0; i < 3; ++i) raw[3 + i] = ev[i] - DV[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) tv[i] = twj[i] - twi[i] - vi[i] * dt - 0.5 * g[i] * dt * dt;
        m3vec(Rbwi, tv, ev);
#pragma unroll
        for (int i = 0; i < 3; ++i) raw[6 + i] = ev[i] - DP[i];
    }
    for (int i = 0; i < 9; ++i) {
        double s = 0.0;
        for (int k = 0; k < 9; ++k) s += sqi[9 * i + k] * raw[k];
        r[i] = s;
    }
    if (!want_jac) return;
    for (int i = 0; i < 108; ++i) J[i] = 0.0;
    // vi: rows 3-5: -S(3:6,3:6) R_bwi ; rows 6-8: -S(6:9,6:9) R_bwi dt ; vj rows 3-5: +S(3:6,3:6) R_bwi
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double a = 0, b = 0;
            for (int k = 0; k < 3; ++k) {
                a += sqi[9 * (3 + i) + 3 + k] * Rbwi[3 * k + j];
                b += sqi[9 * (6 + i) + 6 + k] * Rbwi[3 * k + j];
            }
            J[12 * (3 + i) + j] = -a;
            J[12 * (6 + i) + j] = -b * dt;
            J[12 * (3 + i) + 9 + j] = a;
        }
    // bg: S * [-Jr(-er)^-1 J_Rg ; -J_Vg ; -J_Pg] with er the weighted rotation residual (:1439)
    double mer[3] = {-r[0], -r[1], -r[2]}, Jr[9], Jri[9], A[9];
    double th = nrm3(mer);
    if (th < 1e-6) {
        for (int i = 0; i < 9; ++i) Jr[i] = (i % 4 == 0) ? 1.0 : 0.0;
    } else {
        double P[9], P2[9];
        hat3(mer, P);
        m3mul(P, P, P2);
        double th2 = th * th, a = (1.0 - cos(th)) / th2, b = (th - sin(th)) / (th2 * th);
        for (int i = 0; i < 9; ++i) Jr[i] = -a * P[i] + b * P2[i];
        Jr[0] += 1; Jr[4] += 1; Jr[8] += 1;
    }
    inv3(Jr, Jri);
    m3mul(Jri, JRg, A);
    double T[27], Ta[27];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            T[3 * i + j] = -A[3 * i + j];
            T[3 * (3 + i) + j] = -(double)p.J_Vg[3 * i + j];
            T[3 * (6 + i) + j] = -(double)p.J_Pg[3 * i + j];
            Ta[3 * i + j] = 0.0;
            Ta[3 * (3 + i) + j] = -(double)p.J_Va[3 * i + j];
            Ta[3 * (6 + i) + j] = -(double)p.J_Pa[3 * i + j];
        }
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 3; ++j) {
            double sg = 0, sa = 0;
            for (int k = 0; k < 9; ++k) {
                sg += sqi[9 * i + k] * T[3 * k + j];
                sa += sqi[9 * i + k] * Ta[3 * k + j];
            }
            J[12 * i + 3 + j] = sg;
            J[12 * i + 6 + j] = sa;
        }
}

// sqrt information of an IMU factor (Factors.cpp:1309-1323): chol((cov9 + 1e-8 I)^-1)^T, or I
__device__ __noinline__ void imu_sqrt_info(const vio_preint& p, double* out) {
    double M[9][18];
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 18; ++j)
            M[i][j] = j < 9 ? (double)p.cov9[9 * i + j] + (i == j ? 1e-8 : 0.0) : (j - 9 == i ? 1.0 : 0.0);
    bool ok = true;
    for (int c = 0; c < 9 && ok; ++c) {
        int piv = c;
        for (int rr = c + 1; rr < 9; ++rr)
            if (fabs(M[rr][c]) > fabs(M[piv][c])) piv = rr;
        if (M[piv][c] == 0.0) { ok = false; break; }
        if (piv != c)
            for (int j = 0; j < 18; ++j) { double t = M[c][j]; M[c][j] = M[piv][j]; M[piv][j] = t; }
        double iv = 1.0 / M[c][c];
        for (int j = 0; j < 18; ++j) M[c][j] *= iv;
        for (int rr = 0; rr < 9; ++rr) {
            if (rr == c) continue;
            double f = M[rr][c];
            if (f == 0.0) continue;
            for (int j = 0; j < 18; ++j) M[rr][j] -= f * M[c][j];
        }
    }
    double Lm[81];
    if (ok) {
        for (int i = 0; i < 9; ++i)
            for (int j = 0; j < 9; ++j) Lm[9 * i + j] = M[i][9 + j];
        for (int j = 0; j < 9 && ok; ++j) {
            double d = Lm[9 * j + j];
            for (int k = 0; k < j; ++k) d -= Lm[9 * j + k] * Lm[9 * j + k];
            if (!(d > 0.0)) { ok = false; break; }
            d = sqrt(d);
            Lm[9 * j + j] = d;
            for (int i = j + 1; i < 9; ++i) {
                double s = Lm[9 * i + j];
                for (int k = 0; k < j; ++k) s -= Lm[9 * i + k] * Lm[9 * j + k];
                Lm[9 * i + j] = s / d;
            }
        }
    }
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 9; ++j) out[9 * i + j] = ok ? (j >= i ? Lm[9 * j + i] : 0.0) : (i == j ? 1.0 : 0.0);
}

// ------------------------------------------------------------------------------------------
struct WinCtx {
    const BaWin* w;
    BaWsLayout L;
    const double* pose_raw;
    const uint8_t* kf_const;
    const double* lm_xyz0;
    const uint8_t* lm_var;
    const uint8_t* lm_marg;
    const int32_t* lm_ptr;
    const int32_t* obs_kf;
    const int32_t* obs_lm;
    const float* obs_uv;
    const int32_t* kf_ptr;
    const int32_t* kf_obs;
    const vio_preint* preint;
    const uint8_t* preint_valid;
    const double* vel0;
    double* ws;
    double* sqi;      // [K][81]
    double* Himu;     // [NI_MAX^2]
    double* gimu;     // [NI_MAX]
    uint8_t* outlier; // [N] doubles as the PnP round flags
};

// pose cache for the parameter set at (xp): T_wb = SE3(T_init) * exp(delta), etc.
__device__ void pose_cache(BaShared& sh, const WinCtx& c, const double* xp) {
    int K = c.w->K;
    for (int k = threadIdx.x; k < K; k += BA_THREADS) pose_cache_one(sh.pinit[k], xp + 6 * k, sh.pc[k]);
}

// Evaluate cost (and the Jacobian when want_jac) at the point (xp, xl, xv, xb).
// Returns the total cost of the ACTIVE residual blocks.  Sets sh.st.fail on a PnP evaluation failure.
__device__ double evaluate(BaShared& sh, const WinCtx& c, const double* xp, const double* xl, const double* xv,
                           const double* xb, bool want_jac) {
    const BaWin& w = *c.w;
    const int N = w.N, K = w.K;
    pose_cache(sh, c, xp);
    __syncthreads();
    double cost = 0.0;
    int fail = 0;
    double* r0 = c.ws + c.L.r;
    double* jp = c.ws + c.L.jp;
    double* jl = c.ws + c.L.jl;
    for (int o = threadIdx.x; o < N; o += BA_THREADS) {
        int k = c.obs_kf[o], l = c.obs_lm[o];
        bool active = w.pose_f[k] >= 0 || c.lm_var[l];
        if (!active) continue;
        double Pw[3] = {xl[3 * l], xl[3 * l + 1], xl[3 * l + 2]};
        double r[2], Jp[12], Jl[6];
        bool jzero;
        int f = factor_eval(sh.pc[k], sh.Rcb_raw[k], Pw, (double)c.obs_uv[2 * o], (double)c.obs_uv[2 * o + 1], w.cols,
                            w.rows, w.Lw, c.outlier[o] != 0, w.is_pnp, want_jac, r, Jp, Jl, jzero);
        if (f) { fail = 1; continue; }
        double cst, sc;
        huber(w.huber, r[0] * r[0] + r[1] * r[1], cst, sc);
        cost += cst;
        if (want_jac) {
            r0[o] = r[0] * sc;
            r0[N + o] = r[1] * sc;
#pragma unroll
            for (int i = 0; i < 12; ++i) jp[(int64_t)i * N + o] = jzero ? 0.0 : Jp[i] * sc;
#pragma unroll
            for (int i = 0; i < 6; ++i) jl[(int64_t)i * N + o] = jzero ? 0.0 : Jl[i] * sc;
        }
    }
    if (w.is_vi) {
        for (int k = 1 + threadIdx.x; k < K; k += BA_THREADS) {
            if (!c.preint_valid[k]) continue;
            double r[9];
            imu_eval(c.preint[k], c.sqi + 81 * k, w.gravity, sh.pc[k - 1], sh.pc[k], xv + 3 * (k - 1), xb, xb + 3,
                     xv + 3 * k, want_jac, r, sh.imu_J[k]);
            double sq = 0.0;
            for (int i = 0; i < 9; ++i) {
                sq += r[i] * r[i];
                if (want_jac) sh.imu_r[k][i] = r[i];
            }
            cost += 0.5 * sq;
        }
    }
    double total = block_sum(cost, sh.red);
    double anyfail = block_max((double)fail, sh.redm);
    if (threadIdx.x == 0 && anyfail > 0.0) sh.st.fail = 1;
    __syncthreads();
    return total;
}

// imu-space column map of factor k (12 columns -> imu index or -1)
__device__ __forceinline__ int imu_col(const BaWin& w, int k, int c) {
    int f;
    if (c < 3) f = w.vel_f[k - 1] >= 0 ? w.vel_f[k - 1] + c : -1;
    else if (c < 6) f = w.bg_f >= 0 ? w.bg_f + c - 3 : -1;
    else if (c < 9) f = w.ba_f >= 0 ? w.ba_f + c - 6 : -1;
    else f = w.vel_f[k] >= 0 ? w.vel_f[k] + c - 9 : -1;
    return f < 0 ? -1 : f - w.np;
}

// Normal-equation statistics after a Jacobian evaluation: per-pose U/g, per-landmark V/g,
// IMU H/g; gradient max-norm; column norms (for the Jacobi scaling at iteration 0).
__device__ void linearise(BaShared& sh, const WinCtx& c, bool first) {
    const BaWin& w = *c.w;
    const int N = w.N, K = w.K, L = w.L;
    const double* r0 = c.ws + c.L.r;
    const double* jp = c.ws + c.L.jp;
    const double* jl = c.ws + c.L.jl;
    double gm = 0.0;
    // landmarks
    double* V = c.ws + c.L.V;
    double* gl = c.ws + c.L.gl;
    double* sl = c.ws + c.L.s_l;
    for (int l = threadIdx.x; l < L; l += BA_THREADS) {
        if (!c.lm_var[l]) continue;
        double v[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
        for (int o = c.lm_ptr[l]; o < c.lm_ptr[l + 1]; ++o) {
            double a0 = jl[o], a1 = jl[(int64_t)N + o], a2 = jl[2 * (int64_t)N + o];
            double b0 = jl[3 * (int64_t)N + o], b1 = jl[4 * (int64_t)N + o], b2 = jl[5 * (int64_t)N + o];
            double ra = r0[o], rb = r0[N + o];
            v[0] += a0 * a0 + b0 * b0; v[1] += a0 * a1 + b0 * b1; v[2] += a0 * a2 + b0 * b2;
            v[3] += a1 * a1 + b1 * b1; v[4] += a1 * a2 + b1 * b2; v[5] += a2 * a2 + b2 * b2;
            g[0] += a0 * ra + b0 * rb; g[1] += a1 * ra + b1 * rb; g[2] += a2 * ra + b2 * rb;
        }
        for (int i = 0; i < 6; ++i) V[(int64_t)i * L + l] = v[i];
        for (int i = 0; i < 3; ++i) gl[(int64_t)i * L + l] = g[i];
        gm = fmax(gm, fmax(fabs(g[0]), fmax(fabs(g[1]), fabs(g[2]))));
        if (first) {
            sl[l] = 1.0 / (1.0 + sqrt(v[0]));
            sl[(int64_t)L + l] = 1.0 / (1.0 + sqrt(v[3]));
            sl[2 * (int64_t)L + l] = 1.0 / (1.0 + sqrt(v[5]));
        }
    }
    // poses: one wave per pose, lanes over that pose's observations
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int k = wid; k < K; k += BA_THREADS / 64) {
        if (w.pose_f[k] < 0) continue;
        double acc[27];
#pragma unroll
        for (int i = 0; i < 27; ++i) acc[i] = 0.0;
        for (int q = c.kf_ptr[k] + lane; q < c.kf_ptr[k + 1]; q += 64) {
            int o = c.kf_obs[q];
            double a[6], b[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) { a[i] = jp[(int64_t)i * N + o]; b[i] = jp[(int64_t)(6 + i) * N + o]; }
            double ra = r0[o], rb = r0[N + o];
            int idx = 0;
#pragma unroll
            for (int i = 0; i < 6; ++i)
#pragma unroll
                for (int j = i; j < 6; ++j) acc[idx++] += a[i] * a[j] + b[i] * b[j];
#pragma unroll
            for (int i = 0; i < 6; ++i) acc[21 + i] += a[i] * ra + b[i] * rb;
        }
#pragma unroll
        for (int i = 0; i < 27; ++i) acc[i] = wave_sum(acc[i]);
        if (lane == 0)
            for (int i = 0; i < 27; ++i) sh.U[k][i] = acc[i];
    }
    // IMU: per-factor residual/J already in LDS; assemble imu-space H (global) and g.  Factors are
    // added one after another (fixed order); inside a factor the 12 columns map to distinct entries.
    if (w.is_vi) {
        const int ni = w.ni;
        for (int e = threadIdx.x; e < ni * ni; e += BA_THREADS) c.Himu[e] = 0.0;
        for (int p = threadIdx.x; p < ni; p += BA_THREADS) c.gimu[p] = 0.0;
        __syncthreads();
        for (int k = 1; k < K; ++k) {
            if (!c.preint_valid[k]) continue;
            for (int e = threadIdx.x; e < 144 + 12; e += BA_THREADS) {
                if (e < 144) {
                    int cp = e / 12, cq = e % 12;
                    int p = imu_col(w, k, cp), q = imu_col(w, k, cq);
                    if (p < 0 || q < 0) continue;
                    double h = 0.0;
                    for (int i = 0; i < 9; ++i) h += sh.imu_J[k][12 * i + cp] * sh.imu_J[k][12 * i + cq];
                    c.Himu[p * ni + q] += h;
                } else {
                    int cp = e - 144;
                    int p = imu_col(w, k, cp);
                    if (p < 0) continue;
                    double g = 0.0;
                    for (int i = 0; i < 9; ++i) g += sh.imu_J[k][12 * i + cp] * sh.imu_r[k][i];
                    c.gimu[p] += g;
                }
            }
            __syncthreads();
        }
    }
    __syncthreads();
    // f-space gradient and column norms
    for (int f = threadIdx.x; f < w.nf; f += BA_THREADS) {
        double g, cs;
        if (f < w.np) {
            // find pose owning f
            int k = 0;
            for (int kk = 0; kk < K; ++kk)
                if (w.pose_f[kk] >= 0 && f >= w.pose_f[kk] && f < w.pose_f[kk] + 6) k = kk;
            int i = f - w.pose_f[k];
            g = sh.U[k][21 + i];
            // diag index of (i,i) in the packed upper triangle
            int di = i * 6 - (i * (i - 1)) / 2;
            cs = sh.U[k][di];
        } else {
            int p = f - w.np;
            g = c.gimu[p];
            cs = c.Himu[p * w.ni + p];
        }
        sh.g_f[f] = g;
        sh.colsq_f[f] = cs;
        gm = fmax(gm, fabs(g));
        if (first) sh.s_f[f] = 1.0 / (1.0 + sqrt(cs));
    }
    double gmax = block_max(gm, sh.redm);
    if (threadIdx.x == 0) sh.st.gmax = gmax;
    __syncthreads();
}

// ------------------------------------------------------------------------------------------
// Reduced system before the Schur update (schur_eliminator_impl.h:179-377 E^T E-free part): zero,
// Jacobi-scaled pose blocks U, IMU block, LM diagonal.  Also the panel area of schur_gemm is S
// itself, so this runs after the landmark loop.
__device__ void assemble_S(BaShared& sh, const WinCtx& c) {
    const BaWin& w = *c.w;
    const int nf = w.nf, ls = s_ld(nf), npS = 16 * ((nf + 15) >> 4);
    for (int e = threadIdx.x; e < npS * ls; e += BA_THREADS) sh.S[e] = 0.0;
    __syncthreads();
    for (int f = nf + threadIdx.x; f < npS; f += BA_THREADS) { sh.S[f * ls + f] = 1.0; sh.b[f] = 0.0; }
    for (int e = threadIdx.x; e < 36 * w.K; e += BA_THREADS) {
        const int k = e / 36, ij = e - 36 * k;
        const int pf = sh.posef[k];
        if (pf < 0) continue;
        const int i = ij / 6, j = ij % 6;
        const int a = min(i, j), b = max(i, j);
        const int idx = a * 6 - (a * (a - 1)) / 2 + (b - a);
        sh.S[(pf + i) * ls + pf + j] = sh.U[k][idx] * sh.s_f[pf + i] * sh.s_f[pf + j];
    }
    if (w.is_vi) {
        const int ni = w.ni, np = w.np;
        for (int e = threadIdx.x; e < ni * ni; e += BA_THREADS) {
            int p = e / ni, q = e % ni;
            sh.S[(np + p) * ls + np + q] = c.Himu[e] * sh.s_f[np + p] * sh.s_f[np + q];
        }
    }
    __syncthreads();
    for (int f = threadIdx.x; f < nf; f += BA_THREADS) sh.S[f * ls + f] += sh.D_f[f] * sh.D_f[f];
    __syncthreads();
}

// Schur GEMM: S_pp -= Y W^T and b_p -= Y g over landmark chunks (Y = W~ V~^-1), on
// v_mfma_f64_16x16x4_f64.  Per chunk of LC landmarks, fill lanes (landmark slot, keyframe) write
// their pose's 6 rows of the k-major LDS panels At/Bt (k = 3*landmark + component; the value, or
// zero when the keyframe does not see the landmark).  Each wave owns a fixed set of the
// lower-triangle 16x16 output tiles (the Cholesky reads S on and below the diagonal only) and
// accumulates them over all chunks in registers, the rhs column on the VALU beside it.  The panels
// alias S (assembled afterwards), and the global loads of chunk c+1 (observation index one chunk
// further ahead) are in flight while chunk c runs on the matrix cores.  Fixed per-lane k order and
// a fixed shuffle tree: bitwise reproducible.
using d4 = __attribute__((ext_vector_type(4))) double;

constexpr int BA_PANEL = BA_NF_MAX * (BA_NF_MAX + 1) + BA_STAGE;  // S followed by stage
__host__ __device__ constexpr int schur_ks(int T) { return (T & 1) ? 16 * T : 16 * T + 16; }
__host__ __device__ constexpr int schur_kc(int LC) { return (3 * LC + 3) & ~3; }
__host__ __device__ constexpr int schur_lc(int T) {
    int lc = 1;
    while (2 * schur_kc(lc + 1) * schur_ks(T) <= BA_PANEL && schur_kc(lc + 1) <= BA_GCOL) ++lc;
    return lc;
}

template <int T>
__device__ void schur_gemm(BaShared& sh, const WinCtx& c) {
    const BaWin& w = *c.w;
    const int N = w.N, L = w.L, K = w.K, np = w.np;
    constexpr int KS = schur_ks(T);     // k-row stride (doubles): the 4 k-rows of a fragment hit both bank halves
    constexpr int LCMAX = schur_lc(T);
    constexpr int NT = T * (T + 1) / 2;
    constexpr int TPW = (NT + 3) / 4;   // lower tiles per wave
    constexpr int RPW = (T + 3) / 4;    // rhs row groups per wave
    const int LC = min(LCMAX, BA_THREADS / K);  // landmarks per chunk: one fill lane per (landmark, keyframe)
    const int KC = schur_kc(LC);
    double* At = sh.S;
    double* Bt = sh.S + KC * KS;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r16 = lane & 15, kk = lane >> 4;
    const double* jp = c.ws + c.L.jp;
    const double* jl = c.ws + c.L.jl;
    const double* Vi = c.ws + c.L.Vi;
    const double* gl = c.ws + c.L.gl;
    const double* sl = c.ws + c.L.s_l;
    const int* lk = reinterpret_cast<const int*>(c.ws + c.L.lk);
    int trow[TPW], tcol[TPW];
#pragma unroll
    for (int m = 0; m < TPW; ++m) {
        int t = wid + 4 * m, r = 0;
        if (t >= NT) { trow[m] = -1; tcol[m] = 0; continue; }
        while (t > r) { t -= r + 1; ++r; }
        trow[m] = r; tcol[m] = t;
    }
    d4 acc[TPW];
#pragma unroll
    for (int m = 0; m < TPW; ++m) acc[m] = d4{0.0, 0.0, 0.0, 0.0};
    double bacc[RPW];
#pragma unroll
    for (int q = 0; q < RPW; ++q) bacc[q] = 0.0;

    const int jf = threadIdx.x / K, kf = threadIdx.x - jf * K;
    const int pf = jf < LC ? sh.posef[kf] : -1;
    // prefetch registers: observation of the chunk after next, data of the next chunk
    int o_next = -1;
    double pj[12], lj[6], sv[3], vv[6], gq = 0.0;
    auto load_obs = [&](int l0n) -> int {
        const int l = l0n + jf;
        return (pf >= 0 && l < L) ? lk[16 * l + kf] : -1;
    };
    auto load_data = [&](int l0n, int o) {
        const int l = l0n + jf;
        if (o >= 0) {
#pragma unroll
            for (int i = 0; i < 12; ++i) pj[i] = jp[(int64_t)i * N + o];
#pragma unroll
            for (int i = 0; i < 6; ++i) lj[i] = jl[(int64_t)i * N + o];
#pragma unroll
            for (int i = 0; i < 3; ++i) sv[i] = sl[(int64_t)i * L + l];
#pragma unroll
            for (int i = 0; i < 6; ++i) vv[i] = Vi[(int64_t)i * L + l];
        }
        gq = 0.0;
        if (threadIdx.x < KC) {
            const int lg = l0n + threadIdx.x / 3, cg = threadIdx.x % 3;
            if (lg < min(l0n + LC, L) && c.lm_var[lg]) gq = gl[(int64_t)cg * L + lg] * sl[(int64_t)cg * L + lg];
        }
    };
    for (int e = threadIdx.x; e < 2 * KC * KS; e += BA_THREADS) sh.S[e] = 0.0;
    int o_cur = load_obs(0);
    load_data(0, o_cur);
    o_next = load_obs(LC);
    __syncthreads();
    for (int l0 = 0; l0 < L; l0 += LC) {
        const int l1 = min(l0 + LC, L);
        // ---- fill chunk [l0, l1) from the prefetch registers
        if (threadIdx.x < KC) sh.gcol[threadIdx.x] = gq;
        if (pf >= 0) {
            double Y[6][3], Wv[6][3];
            if (o_cur >= 0) {
                const double b0 = lj[0] * sv[0], b1 = lj[1] * sv[1], b2 = lj[2] * sv[2];
                const double d0 = lj[3] * sv[0], d1 = lj[4] * sv[1], d2 = lj[5] * sv[2];
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    const double sp = sh.s_f[pf + i];
                    const double a = pj[i] * sp, e = pj[6 + i] * sp;
                    const double W0 = a * b0 + e * d0, W1 = a * b1 + e * d1, W2 = a * b2 + e * d2;
                    Wv[i][0] = W0; Wv[i][1] = W1; Wv[i][2] = W2;
                    Y[i][0] = W0 * vv[0] + W1 * vv[1] + W2 * vv[2];
                    Y[i][1] = W0 * vv[1] + W1 * vv[3] + W2 * vv[4];
                    Y[i][2] = W0 * vv[2] + W1 * vv[4] + W2 * vv[5];
                }
            } else {
#pragma unroll
                for (int i = 0; i < 6; ++i)
#pragma unroll
                    for (int cc = 0; cc < 3; ++cc) { Y[i][cc] = 0.0; Wv[i][cc] = 0.0; }
            }
#pragma unroll
            for (int cc = 0; cc < 3; ++cc)
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    At[(3 * jf + cc) * KS + pf + i] = Y[i][cc];
                    Bt[(3 * jf + cc) * KS + pf + i] = Wv[i][cc];
                }
        }
        __syncthreads();
        prof_mark(sh, PF_FILL);
        // ---- prefetch: data of the next chunk, observation index of the one after
        o_cur = o_next;
        if (l1 < L) {
            load_data(l1, o_cur);
            o_next = load_obs(l1 + LC);
        }
        // ---- MFMA over the chunk
        const int nsteps = (3 * (l1 - l0) + 3) >> 2;
        for (int st = 0; st < nsteps; ++st) {
            const int kr = (4 * st + kk) * KS;
#pragma unroll
            for (int m = 0; m < TPW; ++m) {
                if (trow[m] < 0) continue;
                const double a = At[kr + 16 * trow[m] + r16];
                const double b = Bt[kr + 16 * tcol[m] + r16];
                acc[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[m], 0, 0, 0);
            }
            const double g = sh.gcol[4 * st + kk];
#pragma unroll
            for (int q = 0; q < RPW; ++q) {
                const int rg = wid + 4 * q;
                if (rg < T) bacc[q] += At[kr + 16 * rg + r16] * g;
            }
        }
        __syncthreads();
        prof_mark(sh, PF_GEMM);
    }
    assemble_S(sh, c);
    const int ls = s_ld(w.nf);
#pragma unroll
    for (int m = 0; m < TPW; ++m) {
        if (trow[m] < 0) continue;
        const int col = 16 * tcol[m] + r16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 16 * trow[m] + 4 * r + kk;
            if (row < np && col < np) sh.S[row * ls + col] -= acc[m][r];
        }
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        double v = bacc[q];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        const int row = 16 * (wid + 4 * q) + r16;
        if (kk == 0 && wid + 4 * q < T && row < np) sh.b[row] -= v;
    }
    __syncthreads();
}

// Cholesky of S (nf x nf in LDS, padded to nb = ceil(nf/16) 16x16 tiles with an identity tail,
// row stride s_ld(nf)) then solve S y = b (y overwrites b).  Blocked right-looking:
//   (A) wave 0 factors the diagonal tile in registers (lane i = row i, pivots and column entries
//       broadcast with v_readlane) and forms its triangular inverse; Linv_J^T goes to the stage area;
//   (B) panel tiles L_IJ = S_IJ Linv_J^T on v_mfma_f64_16x16x4_f64, one tile per wave at a time;
//   (C) trailing lower tiles S_IK -= L_IJ L_KJ^T on the matrix cores.
// Three workgroup barriers per tile column.  The two triangular solves walk the tile columns with
// one wave (lanes = 16 rows x 4 column groups).  Fixed operation order: bitwise reproducible.
// Returns false (uniformly) when a pivot is not positive (S not positive definite).
__device__ __forceinline__ double readlane_d(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

__device__ __noinline__ bool cholesky_solve(BaShared& sh, int nf) {
    double* S = sh.S;
    double* LB = sh.stage;  // [nb][16 m][16 c] = Linv_J[c][m]
    const int ls = s_ld(nf), nb = (nf + 15) >> 4;
    constexpr int NW = BA_THREADS / 64;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r16 = lane & 15, kk = lane >> 4;
    for (int J = 0; J < nb; ++J) {
        const int c0 = 16 * J;
        // (A) diagonal tile
        if (wid == 0) {
            const int i = r16;
            double d[16], il[16];
            const double* row = S + (c0 + i) * ls + c0;
#pragma unroll
            for (int k = 0; k < 16; ++k) d[k] = row[k];  // k > i: upper triangle, never used
            int bad = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const double piv = readlane_d(d[j], j);
                bad |= !(piv > 0.0);
                const double lj = sqrt(piv);
                il[j] = 1.0 / lj;
                const double cj = i == j ? lj : d[j] * il[j];
                d[j] = cj;
#pragma unroll
                for (int k = j + 1; k < 16; ++k) d[k] -= cj * readlane_d(cj, k);
            }
            // column i of Linv (lower): x[q] = Linv[q][i]
            double x[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                double s = q == i ? 1.0 : 0.0;
#pragma unroll
                for (int m = 0; m < q; ++m) s -= readlane_d(d[m], q) * x[m];
                x[q] = s * il[q];
            }
            // LB[m][c] = Linv[c][m]: lane m holds column m of Linv, i.e. Linv[c][m] = x[c]
            if (kk == 0) {
                double* dst = LB + 256 * J + 16 * i;
#pragma unroll
                for (int q = 0; q < 16; ++q) dst[q] = x[q];
            }
            if (lane == 0) sh.chol_bad = bad;
        }
        __syncthreads();
        if (sh.chol_bad) return false;
        // (B) panel: L_IJ = S_IJ Linv_J^T
        const double* lb = LB + 256 * J;
        for (int I = J + 1 + wid; I < nb; I += NW) {
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            double* A = S + 16 * I * ls + c0;
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const double a = A[r16 * ls + 4 * st + kk];
                const double bb = lb[(4 * st + kk) * 16 + r16];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) A[(kk + 4 * r) * ls + r16] = acc[r];
        }
        __syncthreads();
        // (C) trailing update of the lower tiles (I, K), J < K <= I < nb
        const int m = nb - J - 1, nt = m * (m + 1) / 2;
        for (int t = wid; t < nt; t += NW) {
            int I = 0, tt = t;
            while (tt > I) { tt -= I + 1; ++I; }
            const int Kt = tt + J + 1;
            I += J + 1;
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            const double* Ai = S + 16 * I * ls + c0;
            const double* Bk = S + 16 * Kt * ls + c0;
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const double a = Ai[r16 * ls + 4 * st + kk];
                const double bb = Bk[r16 * ls + 4 * st + kk];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
            }
            double* C = S + 16 * I * ls + 16 * Kt;
#pragma unroll
            for (int r = 0; r < 4; ++r) C[(kk + 4 * r) * ls + r16] -= acc[r];
        }
        __syncthreads();
    }
    // triangular solves by wave 0: lane (row r16 of the tile column, column group kk)
    if (wid == 0) {
        double* y = sh.b;
        for (int J = 0; J < nb; ++J) {  // forward: y_J = Linv_J (b_J - sum_{K<J} L_JK y_K)
            const double* Lr = S + (16 * J + r16) * ls;
            double p0 = 0.0, p1 = 0.0;
            int cix = kk;
            for (; cix + 4 < 16 * J; cix += 8) { p0 += Lr[cix] * y[cix]; p1 += Lr[cix + 4] * y[cix + 4]; }
            if (cix < 16 * J) p0 += Lr[cix] * y[cix];
            double t = p0 + p1;
            t += __shfl_xor(t, 16, 64);
            t += __shfl_xor(t, 32, 64);
            t = y[16 * J + r16] - t;
            const double* lb = LB + 256 * J;
            double v = 0.0;
#pragma unroll
            for (int mm = 0; mm < 16; ++mm) v += lb[16 * mm + r16] * readlane_d(t, mm);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            if (kk == 0) y[16 * J + r16] = v;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        for (int J = nb - 1; J >= 0; --J) {  // backward: x_J = Linv_J^T (y_J - sum_{K>J} L_KJ^T x_K)
            double p0 = 0.0, p1 = 0.0;
            int cix = 16 * (J + 1) + kk;
            const int cend = 16 * nb;
            for (; cix + 4 < cend; cix += 8) {
                p0 += S[cix * ls + 16 * J + r16] * y[cix];
                p1 += S[(cix + 4) * ls + 16 * J + r16] * y[cix + 4];
            }
            if (cix < cend) p0 += S[cix * ls + 16 * J + r16] * y[cix];
            double t = p0 + p1;
            t += __shfl_xor(t, 16, 64);
            t += __shfl_xor(t, 32, 64);
            t = y[16 * J + r16] - t;
            const double* lb = LB + 256 * J;
            double v = 0.0;
#pragma unroll
            for (int mm = 0; mm < 16; ++mm) v += lb[16 * r16 + mm] * readlane_d(t, mm);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            if (kk == 0) y[16 * J + r16] = v;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    __syncthreads();
    return true;
}

// One LM step computation (ComputeTrustRegionStep): returns validity uniformly via sh.st.valid.
__device__ void compute_step(BaShared& sh, const WinCtx& c) {
    const BaWin& w = *c.w;
    const int N = w.N, L = w.L, nf = w.nf;
    const double radius = sh.st.radius;
    const double dmin = 1e-6, dmax = 1e32;
    double* Vi = c.ws + c.L.Vi;
    const double* V = c.ws + c.L.V;
    const double* gl = c.ws + c.L.gl;
    const double* sl = c.ws + c.L.s_l;
    double* yl = c.ws + c.L.y_l;
    int bad = 0;
    // (1) landmark blocks V~ = s V s + D^2, inverse via LLT
    for (int l = threadIdx.x; l < L; l += BA_THREADS) {
        if (!c.lm_var[l]) continue;
        double s[3] = {sl[l], sl[(int64_t)L + l], sl[2 * (int64_t)L + l]};
        double v[6];
        for (int i = 0; i < 6; ++i) v[i] = V[(int64_t)i * L + l];
        double a00 = v[0] * s[0] * s[0], a01 = v[1] * s[0] * s[1], a02 = v[2] * s[0] * s[2];
        double a11 = v[3] * s[1] * s[1], a12 = v[4] * s[1] * s[2], a22 = v[5] * s[2] * s[2];
        a00 += fmin(fmax(a00, dmin), dmax) / radius;
        a11 += fmin(fmax(a11, dmin), dmax) / radius;
        a22 += fmin(fmax(a22, dmin), dmax) / radius;
        // LLT
        if (!(a00 > 0.0)) { bad = 1; continue; }
        double l00 = sqrt(a00), l10 = a01 / l00, l20 = a02 / l00;
        double t11 = a11 - l10 * l10;
        if (!(t11 > 0.0)) { bad = 1; continue; }
        double l11 = sqrt(t11), l21 = (a12 - l20 * l10) / l11;
        double t22 = a22 - l20 * l20 - l21 * l21;
        if (!(t22 > 0.0)) { bad = 1; continue; }
        double l22 = sqrt(t22);
        // inverse of L (lower), then V^-1 = L^-T L^-1
        double i00 = 1.0 / l00, i11 = 1.0 / l11, i22 = 1.0 / l22;
        double i10 = -l10 * i00 * i11, i21 = -l21 * i11 * i22;
        double i20 = -(l20 * i00 + l21 * i10) * i22;
        Vi[l] = i00 * i00 + i10 * i10 + i20 * i20;
        Vi[(int64_t)L + l] = i10 * i11 + i20 * i21;
        Vi[2 * (int64_t)L + l] = i20 * i22;
        Vi[3 * (int64_t)L + l] = i11 * i11 + i21 * i21;
        Vi[4 * (int64_t)L + l] = i21 * i22;
        Vi[5 * (int64_t)L + l] = i22 * i22;
    }
    // (2) f-space: LM diagonal and S/b init
    for (int f = threadIdx.x; f < nf; f += BA_THREADS) {
        double d = sh.colsq_f[f] * sh.s_f[f] * sh.s_f[f];
        d = fmin(fmax(d, dmin), dmax);
        sh.D_f[f] = sqrt(d / radius);
        sh.b[f] = sh.s_f[f] * sh.g_f[f];
    }
    double anybad = block_max((double)bad, sh.redm);
    if (anybad > 0.0) {
        if (threadIdx.x == 0) sh.st.valid = 0;
        __syncthreads();
        return;
    }
    prof_mark(sh, PF_PREP);
    // (3) Schur complement
    if (w.np > 0) {
        switch (w.T) {
            case 1: schur_gemm<1>(sh, c); break;
            case 2: schur_gemm<2>(sh, c); break;
            case 3: schur_gemm<3>(sh, c); break;
            case 4: schur_gemm<4>(sh, c); break;
            case 5: schur_gemm<5>(sh, c); break;
            default: schur_gemm<6>(sh, c); break;
        }
    } else {
        assemble_S(sh, c);
    }
    prof_mark(sh, PF_GEMM);
    // (4) reduced solve
    bool ok = true;
    if (nf > 0) ok = cholesky_solve(sh, nf);
    prof_mark(sh, PF_CHOL);
    if (!ok) {
        if (threadIdx.x == 0) sh.st.valid = 0;
        __syncthreads();
        return;
    }
    // (5) back-substitution for the points: y_l = V~^-1 (g~_l - W~^T y_p)
    const double* jp = c.ws + c.L.jp;
    const double* jl = c.ws + c.L.jl;
    double fin = 0.0;
    for (int l = threadIdx.x; l < L; l += BA_THREADS) {
        if (!c.lm_var[l]) continue;
        double s[3] = {sl[l], sl[(int64_t)L + l], sl[2 * (int64_t)L + l]};
        double rhs[3];
        for (int cc = 0; cc < 3; ++cc) rhs[cc] = gl[(int64_t)cc * L + l] * s[cc];
        for (int o = c.lm_ptr[l]; o < c.lm_ptr[l + 1]; ++o) {
            int pf = w.pose_f[c.obs_kf[o]];
            if (pf < 0) continue;
            double e0 = 0, e1 = 0;  // (Jp s_p) y_p  for both residual rows
            for (int i = 0; i < 6; ++i) {
                double yp = sh.b[pf + i] * sh.s_f[pf + i];
                e0 += jp[(int64_t)i * N + o] * yp;
                e1 += jp[(int64_t)(6 + i) * N + o] * yp;
            }
            for (int cc = 0; cc < 3; ++cc)
                rhs[cc] -= s[cc] * (jl[(int64_t)cc * N + o] * e0 + jl[(int64_t)(3 + cc) * N + o] * e1);
        }
        double vi[6];
        for (int i = 0; i < 6; ++i) vi[i] = Vi[(int64_t)i * L + l];
        double y0 = vi[0] * rhs[0] + vi[1] * rhs[1] + vi[2] * rhs[2];
        double y1 = vi[1] * rhs[0] + vi[3] * rhs[1] + vi[4] * rhs[2];
        double y2 = vi[2] * rhs[0] + vi[4] * rhs[1] + vi[5] * rhs[2];
        yl[l] = y0; yl[(int64_t)L + l] = y1; yl[2 * (int64_t)L + l] = y2;
        if (!isfinite(y0) || !isfinite(y1) || !isfinite(y2)) fin = 1.0;
    }
    for (int f = threadIdx.x; f < nf; f += BA_THREADS)
        if (!isfinite(sh.b[f])) fin = 1.0;
    double nonfinite = block_max(fin, sh.redm);
    if (threadIdx.x == 0) sh.st.valid = nonfinite > 0.0 ? 0 : 1;
    __syncthreads();
    prof_mark(sh, PF_BACKSUB);
}

// delta = -y .* s ; model cost change -(J delta)^T (r + J delta / 2); candidate = x + delta
__device__ void make_candidate(BaShared& sh, const WinCtx& c) {
    const BaWin& w = *c.w;
    const int N = w.N, L = w.L, K = w.K;
    const double* r0 = c.ws + c.L.r;
    const double* jp = c.ws + c.L.jp;
    const double* jl = c.ws + c.L.jl;
    const double* sl = c.ws + c.L.s_l;
    const double* yl = c.ws + c.L.y_l;
    double* ws = c.ws;
    // f-space deltas into sh.D_f (reuse) : delta_f = -y_f * s_f
    for (int f = threadIdx.x; f < w.nf; f += BA_THREADS) sh.D_f[f] = -sh.b[f] * sh.s_f[f];
    __syncthreads();
    double mc = 0.0, sn = 0.0, xn = 0.0;
    for (int o = threadIdx.x; o < N; o += BA_THREADS) {
        int k = c.obs_kf[o], l = c.obs_lm[o];
        int pf = w.pose_f[k];
        bool lv = c.lm_var[l];
        if (pf < 0 && !lv) continue;
        double m0 = 0, m1 = 0;
        if (pf >= 0)
            for (int i = 0; i < 6; ++i) {
                double d = sh.D_f[pf + i];
                m0 += jp[(int64_t)i * N + o] * d;
                m1 += jp[(int64_t)(6 + i) * N + o] * d;
            }
        if (lv)
            for (int cc = 0; cc < 3; ++cc) {
                double d = -yl[(int64_t)cc * L + l] * sl[(int64_t)cc * L + l];
                m0 += jl[(int64_t)cc * N + o] * d;
                m1 += jl[(int64_t)(3 + cc) * N + o] * d;
            }
        mc -= m0 * (r0[o] + m0 / 2.0) + m1 * (r0[N + o] + m1 / 2.0);
    }
    if (w.is_vi) {
        for (int k = 1 + threadIdx.x; k < K; k += BA_THREADS) {
            if (!c.preint_valid[k]) continue;
            double m[9];
            for (int i = 0; i < 9; ++i) m[i] = 0.0;
            for (int cp = 0; cp < 12; ++cp) {
                int p = imu_col(w, k, cp);
                if (p < 0) continue;
                double d = sh.D_f[w.np + p];
                for (int i = 0; i < 9; ++i) m[i] += sh.imu_J[k][12 * i + cp] * d;
            }
            for (int i = 0; i < 9; ++i) mc -= m[i] * (sh.imu_r[k][i] + m[i] / 2.0);
        }
    }
    // candidate and norms (x - candidate computed like Ceres' (x_ - candidate_x_).norm())
    double* xp = ws + c.L.x_pose; double* cp_ = ws + c.L.c_pose;
    double* xl = ws + c.L.x_lm;   double* cl = ws + c.L.c_lm;
    double* xv = ws + c.L.x_vel;  double* cv = ws + c.L.c_vel;
    double* xb = ws + c.L.x_bias; double* cb = ws + c.L.c_bias;
    for (int e = threadIdx.x; e < 6 * K; e += BA_THREADS) {
        int k = e / 6, i = e % 6;
        int pf = w.pose_f[k];
        double x = xp[e];
        double cnd = pf >= 0 ? x + sh.D_f[pf + i] : x;
        cp_[e] = cnd;
        if (pf >= 0) { double d = x - cnd; sn += d * d; xn += cnd * cnd; }
    }
    for (int e = threadIdx.x; e < 3 * L; e += BA_THREADS) {
        int l = e / 3, cc = e % 3;
        double x = xl[e];
        double cnd = c.lm_var[l] ? x + (-yl[(int64_t)cc * L + l] * sl[(int64_t)cc * L + l]) : x;
        cl[e] = cnd;
        if (c.lm_var[l]) { double d = x - cnd; sn += d * d; xn += cnd * cnd; }
    }
    if (w.is_vi) {
        for (int e = threadIdx.x; e < 3 * K; e += BA_THREADS) {
            int k = e / 3, cc = e % 3;
            int vf = w.vel_f[k];
            double x = xv[e];
            double cnd = vf >= 0 ? x + sh.D_f[vf + cc] : x;
            cv[e] = cnd;
            if (vf >= 0) { double d = x - cnd; sn += d * d; xn += cnd * cnd; }
        }
        for (int e = threadIdx.x; e < 6; e += BA_THREADS) {
            int f = e < 3 ? w.bg_f + e : w.ba_f + e - 3;
            bool act = e < 3 ? w.bg_f >= 0 : w.ba_f >= 0;
            double x = xb[e];
            double cnd = act ? x + sh.D_f[f] : x;
            cb[e] = cnd;
            if (act) { double d = x - cnd; sn += d * d; xn += cnd * cnd; }
        }
    }
    double mct = block_sum(mc, sh.red);
    double snt = block_sum(sn, sh.red);
    double xnt = block_sum(xn, sh.red);
    if (threadIdx.x == 0) {
        sh.st.model_change = mct;
        sh.st.step_norm = sqrt(snt);
        sh.st.cand_x_norm2 = xnt;
    }
    __syncthreads();
    prof_mark(sh, PF_CAND);
}

__device__ void accept_candidate(BaShared& sh, const WinCtx& c) {
    const BaWin& w = *c.w;
    double* ws = c.ws;
    const int K = w.K, L = w.L;
    for (int e = threadIdx.x; e < 6 * K; e += BA_THREADS) ws[c.L.x_pose + e] = ws[c.L.c_pose + e];
    for (int e = threadIdx.x; e < 3 * L; e += BA_THREADS) ws[c.L.x_lm + e] = ws[c.L.c_lm + e];
    for (int e = threadIdx.x; e < 3 * K; e += BA_THREADS) ws[c.L.x_vel + e] = ws[c.L.c_vel + e];
    for (int e = threadIdx.x; e < 6; e += BA_THREADS) ws[c.L.x_bias + e] = ws[c.L.c_bias + e];
    __syncthreads();
}

// ------------------------------------------------------------------------------------------
// One ceres::Solve from the current workspace point.  Ceres semantics: see trust_region_minimizer.cc.
__device__ void lm_solve(BaShared& sh, const WinCtx& c) {
    const BaWin& w = *c.w;
    double* ws = c.ws;
    double* xp = ws + c.L.x_pose;
    double* xl = ws + c.L.x_lm;
    double* xv = ws + c.L.x_vel;
    double* xb = ws + c.L.x_bias;
    const bool fixed = w.fixed_iter != 0;
    if (threadIdx.x == 0) {
        LmState& s = sh.st;
        s.radius = 1e4;
        s.decrease_factor = 2.0;
        s.x_norm = -1.0;
        s.min_cost = DBL_MAX;
        s.iteration = 0;
        s.nsucc = s.nunsucc = 0;
        s.consecutive_invalid = 0;
        s.termination = VIO_TERM_NO_CONVERGENCE;
        s.done = 0;
        s.fail = 0;
    }
    __syncthreads();
    // IterationZero
    prof_mark(sh, PF_CTRL);
    double cost = evaluate(sh, c, xp, xl, xv, xb, true);
    prof_mark(sh, PF_EVAL_J);
    if (sh.st.fail) {
        if (threadIdx.x == 0) {
            sh.st.termination = VIO_TERM_FAILURE;
            sh.st.initial_cost = sh.st.fixed_cost;
            sh.st.final_cost = sh.st.fixed_cost;
            sh.st.done = 1;
        }
        __syncthreads();
        return;
    }
    linearise(sh, c, true);
    prof_mark(sh, PF_LIN);
    if (threadIdx.x == 0) {
        LmState& s = sh.st;
        s.x_cost = cost;
        s.initial_cost = cost + s.fixed_cost;
        s.final_cost = s.initial_cost;
        s.step_eval_current = cost;
        s.step_ok = 1;
        s.iter_cost = cost + s.fixed_cost;
    }
    __syncthreads();
    for (;;) {
        // FinalizeIterationAndCheckIfMinimizerCanContinue
        if (threadIdx.x == 0) {
            LmState& s = sh.st;
            if (s.step_ok) {
                s.nsucc++;
                if (s.x_cost < s.min_cost) s.min_cost = s.x_cost;
            } else {
                s.nunsucc++;
            }
            s.final_cost = fmin(s.final_cost, s.iter_cost);
            if (s.iteration >= w.max_iter) { s.termination = VIO_TERM_NO_CONVERGENCE; s.done = 1; }
            else if (!fixed && s.step_ok && s.gmax <= 1e-10) { s.termination = VIO_TERM_CONVERGENCE; s.done = 1; }
            else if (!fixed && s.radius <= 1e-32) { s.termination = VIO_TERM_CONVERGENCE; s.done = 1; }
            if (!s.done) s.iteration++;
        }
        __syncthreads();
        if (sh.st.done) break;
        prof_mark(sh, PF_CTRL);
        compute_step(sh, c);
        bool valid = sh.st.valid;
        if (valid) {
            make_candidate(sh, c);
            if (threadIdx.x == 0) sh.st.valid = sh.st.model_change > 0.0;
            __syncthreads();
            valid = sh.st.valid;
        }
        if (!valid) {
            if (threadIdx.x == 0) {
                LmState& s = sh.st;
                if (++s.consecutive_invalid >= 5) {
                    s.termination = VIO_TERM_FAILURE;
                    s.done = 1;
                } else {
                    s.radius /= s.decrease_factor;
                    s.decrease_factor *= 2.0;
                    s.step_ok = 0;
                    s.iter_cost = s.x_cost + s.fixed_cost;
                }
            }
            __syncthreads();
            if (sh.st.done) break;
            continue;
        }
        if (threadIdx.x == 0) { sh.st.consecutive_invalid = 0; sh.st.fail = 0; }
        __syncthreads();
        prof_mark(sh, PF_CTRL);
        double cc = evaluate(sh, c, ws + c.L.c_pose, ws + c.L.c_lm, ws + c.L.c_vel, ws + c.L.c_bias, false);
        prof_mark(sh, PF_EVAL_C);
        if (threadIdx.x == 0) {
            LmState& s = sh.st;
            s.cand_cost = s.fail ? DBL_MAX : cc;
            s.fail = 0;
            if (!fixed && s.step_norm <= 1e-8 * (s.x_norm + 1e-8)) { s.termination = VIO_TERM_CONVERGENCE; s.done = 1; }
            else if (!fixed && fabs(s.x_cost - s.cand_cost) <= 1e-6 * s.x_cost) { s.termination = VIO_TERM_CONVERGENCE; s.done = 1; }
            else {
                double rel = s.cand_cost >= DBL_MAX ? -DBL_MAX : (s.step_eval_current - s.cand_cost) / s.model_change;
                s.rel = rel;
                s.step_ok = rel > 1e-3;
                if (!s.step_ok) {
                    s.iter_cost = s.cand_cost + s.fixed_cost;
                    s.radius /= s.decrease_factor;
                    s.decrease_factor *= 2.0;
                }
            }
        }
        __syncthreads();
        if (sh.st.done) break;
        if (sh.st.step_ok) {
            accept_candidate(sh, c);
            prof_mark(sh, PF_CTRL);
            double nc = evaluate(sh, c, xp, xl, xv, xb, true);
            prof_mark(sh, PF_EVAL_J);
            if (sh.st.fail) {
                if (threadIdx.x == 0) { sh.st.termination = VIO_TERM_FAILURE; sh.st.done = 1; }
                __syncthreads();
                break;
            }
            linearise(sh, c, false);
            prof_mark(sh, PF_LIN);
            if (threadIdx.x == 0) {
                LmState& s = sh.st;
                s.x_norm = sqrt(s.cand_x_norm2);
                s.x_cost = nc;
                double q = s.rel;
                s.radius = s.radius / fmax(1.0 / 3.0, 1.0 - pow(2.0 * q - 1.0, 3.0));
                s.radius = fmin(1e16, s.radius);
                s.decrease_factor = 2.0;
                s.step_eval_current = s.cand_cost;
                s.iter_cost = nc + s.fixed_cost;
            }
            __syncthreads();
        }
    }
}

// reset the free parameters of the window to their initial values
__device__ void init_params(BaShared& sh, const WinCtx& c, bool poses_only) {
    const BaWin& w = *c.w;
    double* ws = c.ws;
    for (int e = threadIdx.x; e < 6 * w.K; e += BA_THREADS) ws[c.L.x_pose + e] = 0.0;
    if (!poses_only) {
        for (int e = threadIdx.x; e < 3 * w.L; e += BA_THREADS) ws[c.L.x_lm + e] = c.lm_xyz0[e];
        for (int e = threadIdx.x; e < 3 * w.K; e += BA_THREADS) ws[c.L.x_vel + e] = w.is_vi ? c.vel0[e] : 0.0;
        for (int e = threadIdx.x; e < 6; e += BA_THREADS) ws[c.L.x_bias + e] = e < 3 ? w.bg0[e] : w.ba0[e - 3];
    }
    __syncthreads();
}

__global__ void __launch_bounds__(BA_THREADS, 1) ba_window_kernel(BaPools P) {
    extern __shared__ __align__(16) unsigned char smem_raw[];
    BaShared& sh = *reinterpret_cast<BaShared*>(smem_raw);
    const BaWin& w = P.win[blockIdx.x];
    WinCtx c;
    c.w = &w;
    c.L = ba_ws_layout(w.K, w.L, w.N);
    c.pose_raw = P.pose_raw + 24 * w.o_pose;
    c.kf_const = P.kf_const + w.o_pose;
    c.lm_xyz0 = P.lm_xyz0 + 3 * w.o_lm;
    c.lm_var = P.lm_var + w.o_lm;
    c.lm_marg = P.lm_marg + w.o_lm;
    c.lm_ptr = P.lm_ptr + w.o_lmptr;
    c.obs_kf = P.obs_kf + w.o_obs;
    c.obs_lm = P.obs_lm + w.o_obs;
    c.obs_uv = P.obs_uv + 2 * w.o_obs;
    c.kf_ptr = P.kf_ptr + w.o_kfptr;
    c.kf_obs = P.kf_obs + w.o_obs;
    c.preint = P.preint + w.o_pose;
    c.preint_valid = P.preint_valid + w.o_pose;
    c.vel0 = P.vel0 + 3 * w.o_pose;
    c.ws = P.ws + w.o_ws;
    c.sqi = c.ws + c.L.total;
    c.Himu = c.sqi + 81 * BA_KMAX;
    c.gimu = c.Himu + NI_MAX * NI_MAX;
    c.outlier = P.out_u8 + w.o_obs;
    const int K = w.K, L = w.L, N = w.N;
    if (threadIdx.x == 0) {
        sh.prof_on = P.prof != nullptr;
        for (int i = 0; i < 16; ++i) sh.prof_acc[i] = 0;
        sh.prof_last = __builtin_amdgcn_s_memtime();
    }
    __syncthreads();

    // ---- setup: projected input rotations (SE3d(T_wb_init), SE3d(T_cb)), raw R_cb, IMU sqrt-info
    for (int k = threadIdx.x; k < K; k += BA_THREADS) {
        const double* pr = c.pose_raw + 24 * k;
        polar3(pr, sh.pinit[k]);
        for (int i = 0; i < 3; ++i) sh.pinit[k][9 + i] = pr[9 + i];
        polar3(pr + 12, sh.pinit[k] + 12);
        for (int i = 0; i < 3; ++i) sh.pinit[k][21 + i] = pr[21 + i];
        for (int i = 0; i < 9; ++i) sh.Rcb_raw[k][i] = pr[12 + i];
        if (w.is_vi && k >= 1 && c.preint_valid[k]) imu_sqrt_info(c.preint[k], c.sqi + 81 * k);
    }
    for (int o = threadIdx.x; o < N; o += BA_THREADS) c.outlier[o] = 0;
    for (int k = threadIdx.x; k < BA_KMAX; k += BA_THREADS) sh.posef[k] = k < K ? w.pose_f[k] : -1;
    {   // (landmark, keyframe) -> observation table for the Schur fill (pairs are unique: host-checked)
        int* lk = reinterpret_cast<int*>(c.ws + c.L.lk);
        for (int e = threadIdx.x; e < 16 * L; e += BA_THREADS) lk[e] = -1;
        __syncthreads();
        for (int o = threadIdx.x; o < N; o += BA_THREADS)
            if (c.lm_var[c.obs_lm[o]]) lk[16 * c.obs_lm[o] + c.obs_kf[o]] = o;
    }
    init_params(sh, c, false);

    // ---- fixed cost: residual blocks whose parameters are all constant (program.cc:305-390)
    {
        pose_cache(sh, c, c.ws + c.L.x_pose);
        __syncthreads();
        double fc = 0.0;
        for (int o = threadIdx.x; o < N; o += BA_THREADS) {
            int k = c.obs_kf[o], l = c.obs_lm[o];
            if (w.pose_f[k] >= 0 || c.lm_var[l]) continue;
            double Pw[3] = {c.lm_xyz0[3 * l], c.lm_xyz0[3 * l + 1], c.lm_xyz0[3 * l + 2]};
            double r[2], Jp[12], Jl[6];
            bool jz;
            if (factor_eval(sh.pc[k], sh.Rcb_raw[k], Pw, (double)c.obs_uv[2 * o], (double)c.obs_uv[2 * o + 1], w.cols,
                            w.rows, w.Lw, false, w.is_pnp, false, r, Jp, Jl, jz) == 0) {
                double cst, sc;
                huber(w.huber, r[0] * r[0] + r[1] * r[1], cst, sc);
                fc += cst;
            }
        }
        double fct = block_sum(fc, sh.red);
        if (threadIdx.x == 0) sh.st.fixed_cost = fct;
        __syncthreads();
    }
    prof_mark(sh, PF_SETUP);

    int32_t* si = P.out_i32 + SI_COUNT * blockIdx.x;
    double* sd = P.out_sum + SD_COUNT * blockIdx.x;
    const BaOutLayout OL = ba_out_layout(K, L, N);
    double* out = P.out + w.o_out;

    if (w.is_pnp) {
        int nin = 0, nout = 0;
        double init_cost = 0.0, fin_cost = 0.0;
        int iters = 0, nsu = 0, nun = 0, term = VIO_TERM_CONVERGENCE;
        for (int round = 0; round < w.rounds; ++round) {
            init_params(sh, c, true);
            lm_solve(sh, c);
            if (sh.st.termination == VIO_TERM_FAILURE) init_params(sh, c, true);
            // chi2 + outlier flags (Optimizer.cpp:215-244)
            pose_cache(sh, c, c.ws + c.L.x_pose);
            __syncthreads();
            double inl = 0.0, cin = 0.0, cout_ = 0.0;
            for (int o = threadIdx.x; o < N; o += BA_THREADS) {
                int k = c.obs_kf[o], l = c.obs_lm[o];
                double Pw[3] = {c.lm_xyz0[3 * l], c.lm_xyz0[3 * l + 1], c.lm_xyz0[3 * l + 2]};
                double ch = factor_chi2(sh.pc[k], Pw, (double)c.obs_uv[2 * o], (double)c.obs_uv[2 * o + 1], w.cols, w.rows,
                                        w.info, c.outlier[o] != 0, true);
                bool is_out = !c.lm_marg[l] && ch > w.chi2_thr;
                out[OL.chi2 + o] = ch;
                c.outlier[o] = is_out;
                if (is_out) cout_ += 1.0;
                else { cin += 1.0; inl += ch; }
            }
            double tin = block_sum(cin, sh.red);
            double tout = block_sum(cout_, sh.red);
            double tinl = block_sum(inl, sh.red);
            if (round == 0) init_cost = sh.st.initial_cost;
            iters += sh.st.nsucc + sh.st.nunsucc;
            nsu += sh.st.nsucc;
            nun += sh.st.nunsucc;
            term = sh.st.termination;
            nin = (int)tin;
            nout = (int)tout;
            fin_cost = nin > 0 ? tinl / nin : sh.st.final_cost;
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            si[SI_SUCCESS] = (term != VIO_TERM_FAILURE) && nin >= 10;
            si[SI_TERM] = term;
            si[SI_ITERS] = iters;
            si[SI_NSUCC] = nsu;
            si[SI_NUNSUCC] = nun;
            si[SI_NIN] = nin;
            si[SI_NOUT] = nout;
            si[SI_NBAD] = 0;
            sd[SD_INIT] = init_cost;
            sd[SD_FINAL] = fin_cost;
            sd[SD_FIXED] = 0.0;
        }
        for (int l = threadIdx.x; l < L; l += BA_THREADS) P.out_bad[w.o_lm + l] = 0;
    } else {
        bool any_free = w.nf > 0;
        if (!any_free) {
            for (int l = 0; l < L && !any_free; ++l) any_free = c.lm_var[l];
        }
        if (any_free) {
            lm_solve(sh, c);
            if (sh.st.termination == VIO_TERM_FAILURE) init_params(sh, c, false);
        } else if (threadIdx.x == 0) {
            sh.st.termination = VIO_TERM_CONVERGENCE;
            sh.st.initial_cost = sh.st.final_cost = sh.st.fixed_cost;
            sh.st.nsucc = sh.st.nunsucc = 0;
        }
        __syncthreads();
        // chi2 / outliers / bad landmarks (Optimizer.cpp:425-456, 888-928)
        pose_cache(sh, c, c.ws + c.L.x_pose);
        __syncthreads();
        const double* xl = c.ws + c.L.x_lm;
        double cin = 0.0, cout_ = 0.0, cbad = 0.0;
        for (int l = threadIdx.x; l < L; l += BA_THREADS) {
            int li = 0, lo = 0;
            for (int o = c.lm_ptr[l]; o < c.lm_ptr[l + 1]; ++o) {
                int k = c.obs_kf[o];
                double Pw[3] = {xl[3 * l], xl[3 * l + 1], xl[3 * l + 2]};
                double ch = factor_chi2(sh.pc[k], Pw, (double)c.obs_uv[2 * o], (double)c.obs_uv[2 * o + 1], w.cols, w.rows,
                                        w.info, false, false);
                bool is_out = ch > w.chi2_thr;
                out[OL.chi2 + o] = ch;
                c.outlier[o] = is_out;
                if (is_out) lo++; else li++;
            }
            bool bad = !c.lm_marg[l] && li == 0 && lo >= 2;
            P.out_bad[w.o_lm + l] = bad;
            cin += li;
            cout_ += lo;
            cbad += bad;
        }
        double tin = block_sum(cin, sh.red);
        double tout = block_sum(cout_, sh.red);
        double tbad = block_sum(cbad, sh.red);
        if (threadIdx.x == 0) {
            si[SI_SUCCESS] = sh.st.termination != VIO_TERM_FAILURE;
            si[SI_TERM] = sh.st.termination;
            si[SI_ITERS] = sh.st.nsucc + sh.st.nunsucc;
            si[SI_NSUCC] = sh.st.nsucc;
            si[SI_NUNSUCC] = sh.st.nunsucc;
            si[SI_NIN] = (int)tin;
            si[SI_NOUT] = (int)tout;
            si[SI_NBAD] = (int)tbad;
            sd[SD_INIT] = sh.st.initial_cost;
            sd[SD_FINAL] = sh.st.final_cost;
            sd[SD_FIXED] = sh.st.fixed_cost;
        }
    }
    // ---- outputs: poses T_wb = SE3(T_init) exp(delta), points, velocities, biases
    for (int k = threadIdx.x; k < K; k += BA_THREADS) {
        for (int i = 0; i < 9; ++i) out[OL.T_wb + 12 * k + i] = sh.pc[k][i];
        for (int i = 0; i < 3; ++i) out[OL.T_wb + 12 * k + 9 + i] = sh.pc[k][9 + i];
    }
    for (int e = threadIdx.x; e < 3 * L; e += BA_THREADS) out[OL.lm + e] = c.ws[c.L.x_lm + e];
    for (int e = threadIdx.x; e < 3 * K; e += BA_THREADS) out[OL.vel + e] = c.ws[c.L.x_vel + e];
    for (int e = threadIdx.x; e < 6; e += BA_THREADS) out[OL.bias + e] = c.ws[c.L.x_bias + e];
    __syncthreads();
    prof_mark(sh, PF_POST);
    if (P.prof && threadIdx.x < 16) P.prof[16 * blockIdx.x + threadIdx.x] = sh.prof_acc[threadIdx.x];
}

size_t ba_shared_bytes() { return sizeof(BaShared); }
size_t ba_ws_extra_doubles() { return 81 * BA_KMAX + NI_MAX * NI_MAX + NI_MAX + 32; }

hipError_t launch_ba_windows(const BaPools& P, int n, hipStream_t stream) {
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)ba_window_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)sizeof(BaShared));
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    hipLaunchKernelGGL(ba_window_kernel, dim3(n), dim3(BA_THREADS), sizeof(BaShared), stream, P);
    return hipGetLastError();
}

}  // namespace vio360
