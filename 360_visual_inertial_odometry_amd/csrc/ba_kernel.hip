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

#include <algorithm>
#include <atomic>
#include <mutex>

#include "ba_types.h"
#include "ba_global.h"
#include "ba_factor_dev.h"
#include "chol_dev.h"
#include "lie_dev.h"

namespace vio360 {

#ifndef VIO_BA_CLUSTER_TU
uint64_t ba_layout_sig_ba_kernel() { return ba_layout_sig(); }
uint64_t gba_layout_sig_ba_kernel() { return gba_layout_sig(); }
#else
uint64_t ba_layout_sig_ba_cluster() { return ba_layout_sig(); }
#endif

constexpr int NI_MAX = 3 * VI_KMAX + 6;
// per-window workspace after ba_ws_layout(): IMU sqrt-information, imu-space H and g
__host__ __device__ constexpr int64_t ba_ws_extra() { return 81 * BA_KMAX + NI_MAX * NI_MAX + NI_MAX + 32; }

struct LmState {
    double radius, decrease_factor;
    double x_cost, cand_cost, min_cost, model_change, x_norm, gmax;
    double initial_cost, final_cost, fixed_cost, iter_cost, step_eval_current;
    double step_norm, cand_x_norm2, rel;
    double fused_cost;           // cost at the candidate, evaluated inside compute_step
    // IterationSummary fields of the iteration in progress (pushed to the trace at finalisation)
    double tr_cost_change, tr_step_norm, tr_rel, tr_model;
    int tr_valid, tr_n;
    int iteration, nsucc, nunsucc, consecutive_invalid;
    int termination, done, step_ok, valid, fail, need_jac, pnp_round, cand_fail;
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
    double redv[(BA_THREADS / 64) * 8];  // block_reduce exchange (up to 8 values)
    LmState st;
    unsigned long long prof_acc[VIO_BA_PROF_SLOTS];
    unsigned long long prof_last;
    int prof_on;
    int chol_bad;
    int posef[BA_KMAX];          // copy of BaWin::pose_f (per-lane indexed in the Schur fill)
    int pvalid[BA_KMAX];         // preint_valid
    int8_t icol[BA_KMAX][12];    // imu_col(w, k, c): imu-space index of column c of IMU factor k, or -1
    double Rlin[BA_KMAX][9];     // R_bw at the linearisation point (Jacobians are stored compressed)
};
static_assert(sizeof(BaShared) <= 160 * 1024, "BaShared exceeds the 160 KB LDS of a gfx950 CU");
static_assert(offsetof(BaShared, stage) == offsetof(BaShared, S) + sizeof(double) * BA_NF_MAX * (BA_NF_MAX + 1),
              "Schur panels span S and stage contiguously");

// row stride of S: tile-padded size, odd (conflict-free column walks)
__host__ __device__ constexpr int s_ld(int nf) { return (16 * ((nf + 15) >> 4)) | 1; }
static_assert(16 * ((BA_NF_MAX + 15) >> 4) * s_ld(BA_NF_MAX) <= BA_NF_MAX * (BA_NF_MAX + 1), "S padding");
static_assert(256 * (((BA_NF_MAX + 15) >> 4) + 1) + 16 <= BA_STAGE, "Cholesky tiles (Linv, L of the diagonal tile, rhs) fit the stage area");

// per-phase shader-clock accounting (diagnostic; enabled when BaPools::prof != nullptr)
enum { PF_SETUP = 0, PF_EVAL_J, PF_LIN, PF_PREP, PF_GEMM, PF_CHOL, PF_BACKSUB, PF_CAND, PF_EVAL_C, PF_CTRL, PF_POST, PF_FILL, PF_PFX, PF_ASM, PF_IMU, PF_IMUH,
       PF_EV_F, PF_EV_L, PF_BS_J, PF_BS_L, PF_BS_C, PF_NSLOT = VIO_BA_PROF_SLOTS };
// per-chunk marks inside the walks (PF_EV_*, PF_BS_*) cost a few percent: compiled in on demand
constexpr bool kProfWalk = false;
__device__ __forceinline__ void prof_mark(BaShared& sh, int slot) {
    if (sh.prof_on && threadIdx.x == 0) {
        unsigned long long t = __builtin_amdgcn_s_memtime();
        sh.prof_acc[slot] += t - sh.prof_last;
        sh.prof_last = t;
    }
}

// ------------------------------------------------------------------------------------------
// wave index as a wave-uniform (scalar) value: branches on it stay scalar
static_assert(BA_THREADS >= 192 && BA_KMAX <= 64, "setup runs three per-keyframe jobs on waves 0..2");
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

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

// NS sums then NM maxima of per-thread values over the workgroup in one exchange (two barriers for
// all of them); each value reduced in the fixed order of block_sum / block_max.  red: NW*(NS+NM) doubles
template <int NS, int NM>
__device__ __forceinline__ void block_reduce(double (&v)[NS + NM], double* red) {
    constexpr int NV = NS + NM, NW = BA_THREADS / 64;
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = i < NS ? wave_sum(v[i]) : wave_max(v[i]);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) red[(threadIdx.x >> 6) * NV + i] = v[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        double r = 0.0;
#pragma unroll
        for (int w = 0; w < NW; ++w) r = i < NS ? r + red[w * NV + i] : fmax(r, red[w * NV + i]);
        v[i] = r;
    }
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
__device__ __forceinline__ void imu_eval_inl(const vio_preint& p, const double* sqi, const double* g, const double* pci,
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
__device__ __noinline__ void imu_eval(const vio_preint& p, const double* sqi, const double* g, const double* pci,
                                const double* pcj, const double* vi, const double* bg, const double* ba,
                                const double* vj, bool want_jac, double* r, double* J) {
    imu_eval_inl(p, sqi, g, pci, pcj, vi, bg, ba, vj, want_jac, r, J);
}

// imu_eval with Jacobians by one whole wave: every lane evaluates the factor's common part (bias
// correction, raw residual, the weighted rotation residual and Jr^-1 J_Rg), lane i < 9 returns residual
// row i in r, lane j < 12 writes Jacobian column j (J row-major 9x12, [vi | bg | ba | vj]).  Each output
// element goes through imu_eval's operations in imu_eval's order (same values); the serial chain of
// 486 + 81 dependent multiply-adds becomes 9 + 9 per lane.
__device__ __forceinline__ void imu_eval_wave_inl(const vio_preint& p, const double* sqi, const double* g, const double* pci,
                                           const double* pcj, const double* vi, const double* bg, const double* ba,
                                           const double* vj, int lane, double& r_out, double* J) {
    const double* Rwj = pcj;
    const double* twi = pci + 9;
    const double* twj = pcj + 9;
    const double* Rbwi = pci + 12;
    const double dt = p.dt_total;
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
        m3tmul(DR, Rbwi, A);
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
    // residual rows 0..2 on every lane (the bias Jacobian needs them), row `lane` on lanes < 9
    double r3[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 9; ++k) s += sqi[9 * i + k] * raw[k];
        r3[i] = s;
    }
    {
        const int ri = lane < 9 ? lane : 0;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 9; ++k) s += sqi[9 * ri + k] * raw[k];
        r_out = s;
    }
    if (lane >= 12) return;
    // column `col` of J written row by row (the rows of the sqrt-information read as they are used: the
    // function stays within the 128 registers of its callers' 4-waves-per-SIMD bound, no scratch)
    const int col = lane;
    if (col < 3 || col >= 9) {  // vi (col 0..2) / vj (col 9..11): diagonal sqrt-information blocks only
        const int j = col < 3 ? col : col - 9;
#pragma unroll
        for (int i = 0; i < 3; ++i) J[12 * i + col] = 0.0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            double a = 0, b = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                a += sqi[9 * (3 + i) + 3 + k] * Rbwi[3 * k + j];
                b += sqi[9 * (6 + i) + 6 + k] * Rbwi[3 * k + j];
            }
            J[12 * (3 + i) + col] = col < 3 ? -a : a;
            J[12 * (6 + i) + col] = col < 3 ? -b * dt : 0.0;
        }
    } else {  // bg (col 3..5) / ba (col 6..8)
        const int j = col < 6 ? col - 3 : col - 6;
        double Tc[9];  // column j of T (bg) or Ta (ba)
        if (col < 6) {
            double mer[3] = {-r3[0], -r3[1], -r3[2]}, Jr[9], Jri[9], A[9];
            double th = nrm3(mer);
            if (th < 1e-6) {
#pragma unroll
                for (int i = 0; i < 9; ++i) Jr[i] = (i % 4 == 0) ? 1.0 : 0.0;
            } else {
                double P[9], P2[9];
                hat3(mer, P);
                m3mul(P, P, P2);
                double th2 = th * th, a = (1.0 - cos(th)) / th2, b = (th - sin(th)) / (th2 * th);
#pragma unroll
                for (int i = 0; i < 9; ++i) Jr[i] = -a * P[i] + b * P2[i];
                Jr[0] += 1; Jr[4] += 1; Jr[8] += 1;
            }
            inv3(Jr, Jri);
            m3mul(Jri, JRg, A);
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                Tc[i] = -A[3 * i + j];
                Tc[3 + i] = -(double)p.J_Vg[3 * i + j];
                Tc[6 + i] = -(double)p.J_Pg[3 * i + j];
            }
        } else {
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                Tc[i] = 0.0;
                Tc[3 + i] = -(double)p.J_Va[3 * i + j];
                Tc[6 + i] = -(double)p.J_Pa[3 * i + j];
            }
        }
#pragma unroll 1
        for (int i = 0; i < 9; ++i) {
            double s = 0;
#pragma unroll
            for (int k = 0; k < 9; ++k) s += sqi[9 * i + k] * Tc[k];
            J[12 * i + col] = s;
        }
    }
}
__device__ __noinline__ void imu_eval_wave(const vio_preint& p, const double* sqi, const double* g, const double* pci,
                                           const double* pcj, const double* vi, const double* bg, const double* ba,
                                           const double* vj, int lane, double& r_out, double* J) {
    imu_eval_wave_inl(p, sqi, g, pci, pcj, vi, bg, ba, vj, lane, r_out, J);
}

// InertialFactorFixedGravity ctor (Factors.cpp:1310-1323): sqrt-information = chol((cov + 1e-8 I)^-1)^T,
// identity when the inverse or its Cholesky fails.  One whole wave per factor: Gauss-Jordan with
// partial pivoting on [Sigma | I] with lane j < 18 holding column j (9 rows in registers, pivot row
// and multipliers broadcast by v_readlane), then the Cholesky of the inverse with lane i < 9 holding
// row i.  Every matrix element goes through the same operations in the same order as the serial
// elimination (oracle/ba_oracle.c), so the result is the same; nothing is dynamically indexed.
__device__ __forceinline__ void imu_sqrt_info_wave_inl(const vio_preint& p, double* out) {
    const int lane = threadIdx.x & 63;
    const int j = lane < 18 ? lane : 17;
    double m[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) m[i] = j < 9 ? (double)p.cov9[9 * i + j] + (i == j ? 1e-8 : 0.0) : (j - 9 == i ? 1.0 : 0.0);
    bool ok = true;
#pragma unroll
    for (int c = 0; c < 9; ++c) {
        if (!ok) break;
        // pivot row: the largest |M[r][c]|, r >= c, first one on ties (lane c scans its column)
        int pv = c;
        double bv = fabs(m[c]), pval = m[c];
#pragma unroll
        for (int rr = c + 1; rr < 9; ++rr)
            if (fabs(m[rr]) > bv) { bv = fabs(m[rr]); pv = rr; pval = m[rr]; }
        const int piv = __builtin_amdgcn_readlane(pv, c);
        if (readlane_d(pval, c) == 0.0) { ok = false; break; }
#pragma unroll
        for (int rr = c + 1; rr < 9; ++rr)
            if (rr == piv) { const double t = m[c]; m[c] = m[rr]; m[rr] = t; }
        const double iv = 1.0 / readlane_d(m[c], c);
        m[c] *= iv;
#pragma unroll
        for (int rr = 0; rr < 9; ++rr) {
            if (rr == c) continue;
            const double f = readlane_d(m[rr], c);
            if (f == 0.0) continue;
            m[rr] -= f * m[c];
        }
    }
    // row i of the inverse into lane i: Inv[i][k] = M[i][9 + k] (lane 9 + k, register i)
    double r[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        r[k] = 0.0;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const double v = readlane_d(m[i], 9 + k);
            if (lane == i) r[k] = v;
        }
    }
    if (ok) {
#pragma unroll
        for (int c = 0; c < 9; ++c) {
            double d = r[c];  // meaningful on lane c: L[c][c] - sum_k L[c][k]^2
#pragma unroll
            for (int k = 0; k < c; ++k) d -= r[k] * r[k];
            const double dc = readlane_d(d, c);
            if (!(dc > 0.0)) { ok = false; break; }
            const double sd = sqrt(dc);
            double s = r[c];
#pragma unroll
            for (int k = 0; k < c; ++k) s -= r[k] * readlane_d(r[k], c);
            if (lane == c) r[c] = sd;
            else if (lane > c && lane < 9) r[c] = s / sd;
        }
    }
    // out (row-major, upper) = L^T: lane jj writes column jj, out[i][jj] = L[jj][i] for i <= jj
    if (lane < 9) {
#pragma unroll
        for (int i = 0; i < 9; ++i)
            out[9 * i + lane] = ok ? (i <= lane ? r[i] : 0.0) : (i == lane ? 1.0 : 0.0);
    }
}
__device__ __noinline__ void imu_sqrt_info_wave(const vio_preint& p, double* out) {
    imu_sqrt_info_wave_inl(p, out);
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
    vio_ba_iteration* trace;  // [w.tr_cap] Summary::iterations
};

// Summary::iterations: FinalizeIterationAndCheckIfMinimizerCanContinue pushes the iteration summary
// (trust_region_minimizer.cc:313-348); one lane
__device__ inline void trace_push(const WinCtx& c, LmState& s) {
    if (s.tr_n < c.w->tr_cap) {
        vio_ba_iteration& t = c.trace[s.tr_n];
        t.iteration = s.iteration;
        t.step_is_valid = s.tr_valid;
        t.step_is_successful = s.step_ok;
        t._pad = 0;
        t.cost = s.iter_cost;
        t.cost_change = s.tr_cost_change;
        t.gradient_max_norm = s.gmax;
        t.step_norm = s.tr_step_norm;
        t.relative_decrease = s.tr_rel;
        t.trust_region_radius = s.radius;
        t.model_cost_change = s.tr_model;
    }
    s.tr_n++;
}
// a new iteration's summary: zero-length, invalid until the step says otherwise (IterationSummary())
__device__ inline void trace_begin(LmState& s) {
    s.tr_valid = 0;
    s.tr_cost_change = s.tr_step_norm = s.tr_rel = s.tr_model = 0.0;
}
// Ceres' gradient max norm term |x - Plus(x, -g)| (trust_region_minimizer.cc:288-299; no local
// parameterization: Plus is x + delta) — |g| up to the roundoff of x - g
__device__ __forceinline__ double grad_term(double x, double g) { return fabs(x - (x + (-g))); }

// pose cache for the parameter set at (xp): T_wb = SE3(T_init) * exp(delta), etc.
__device__ __forceinline__ void pose_cache(BaShared& sh, const WinCtx& c, const double* xp) {
    int K = c.w->K;
    for (int k = threadIdx.x; k < K; k += BA_THREADS) pose_cache_one(sh.pinit[k], xp + 6 * k, sh.pc[k]);
}

// Compressed observation Jacobian (Factors.cpp:481-534): J_pose = [-A | A [Pb]x], J_point = A R_bw with
// A = sqrt(rho') Jw R_cb (2x3, weighted and Huber-scaled) and Pb the point in the body frame, so the
// workspace keeps 9 doubles per observation (A, Pb) instead of 18; R_bw comes from the pose (LDS).
__device__ __forceinline__ void jac_from_ap(const double* A, const double* Pb, const double* Rbw, double* Jp,
                                            double* Jl) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const double* a = A + 3 * i;
        Jp[6 * i + 0] = -a[0];
        Jp[6 * i + 1] = -a[1];
        Jp[6 * i + 2] = -a[2];
        Jp[6 * i + 3] = a[1] * Pb[2] - a[2] * Pb[1];
        Jp[6 * i + 4] = a[2] * Pb[0] - a[0] * Pb[2];
        Jp[6 * i + 5] = a[0] * Pb[1] - a[1] * Pb[0];
#pragma unroll
        for (int j = 0; j < 3; ++j) Jl[3 * i + j] = a[0] * Rbw[j] + a[1] * Rbw[3 + j] + a[2] * Rbw[6 + j];
    }
}

// Landmark-chunk walker: lane (jf, kf) = (landmark slot, keyframe) of a chunk of LC = BA_THREADS/K
// landmarks; its observation is lk[16 l + kf] (or -1).  A landmark's observations are contiguous in
// the landmark-sorted SoA arrays, so consecutive lanes touch consecutive observations (coalesced),
// a lane keeps one keyframe (its pose cache / pose sums) for the whole walk, and landmark sums are
// fixed-order reductions over the K lanes of a slot through LDS.
struct Walk {
    int LC, jf, kf;
    bool on;
};
__device__ __forceinline__ Walk walk_geom(int K) {
    Walk g;
    const int k = K > 0 ? K : 1;
    g.LC = BA_THREADS / k;
    g.jf = threadIdx.x / k;
    g.kf = threadIdx.x - g.jf * k;
    g.on = K > 0 && g.jf < g.LC;
    return g;
}

// Landmark sums of one walk chunk: q[i][slot*K + kf] (i < 9: the 6 V~ entries and 3 gradient entries
// of each observation lane) summed over the K keyframe lanes of each landmark slot, kf ascending.
// One lane per (entry, landmark) pair: a 9xLC job instead of LC lanes summing 9K values each.
// Writes V / g_l (and the Jacobi scaling s_l on the first linearisation); returns the lane's
// running max |g_l| (combined by a block max later, exact in any order).
__device__ __forceinline__ double lm_sums9(const double* q, int l0, const Walk& g, int K, int L,
                                           const uint8_t* lm_var, const double* xl, double* V, double* gl, double* sl,
                                           bool first, double gm) {
    for (int t = threadIdx.x; t < 9 * g.LC; t += BA_THREADS) {
        const int i = t / g.LC, j = t - i * g.LC, lj = l0 + j;
        if (lj >= L || !lm_var[lj]) continue;
        const double* src = q + i * BA_THREADS + j * K;
        double v = 0.0;
#pragma unroll
        for (int kf = 0; kf < BA_KMAX; ++kf)
            if (kf < K) v += src[kf];
        if (i < 6) {
            V[(int64_t)i * L + lj] = v;
        } else {
            gl[(int64_t)(i - 6) * L + lj] = v;
            gm = fmax(gm, grad_term(xl[3 * lj + i - 6], v));
        }
        if (first && (i == 0 || i == 3 || i == 5)) sl[(int64_t)(i == 0 ? 0 : i == 3 ? 1 : 2) * L + lj] = 1.0 / (1.0 + sqrt(v));
    }
    return gm;
}

// IMU factors (one lane per factor): cost, and residual/Jacobian into LDS when want_jac
__device__ __forceinline__ double imu_factors(BaShared& sh, const WinCtx& c, const double* xv, const double* xb, bool want_jac) {
    const BaWin& w = *c.w;
    double cost = 0.0;
    if (!w.is_vi) return 0.0;
    for (int k = 1 + threadIdx.x; k < w.K; k += BA_THREADS) {
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
    return cost;
}

__device__ __forceinline__ void lin_tail(BaShared& sh, const WinCtx& c, bool first, double gm, const double* xp,
                                         const double* xv, const double* xb);

// value of reduced-system parameter f (pose delta, velocity or bias component) at (xp, xv, xb)
__device__ inline double f_param_value(const BaWin& w, int f, const double* xp, const double* xv, const double* xb) {
    for (int k = 0; k < w.K; ++k) {
        if (w.pose_f[k] >= 0 && f >= w.pose_f[k] && f < w.pose_f[k] + 6) return xp[6 * k + f - w.pose_f[k]];
        if (w.vel_f[k] >= 0 && f >= w.vel_f[k] && f < w.vel_f[k] + 3) return xv[3 * k + f - w.vel_f[k]];
    }
    if (w.bg_f >= 0 && f >= w.bg_f && f < w.bg_f + 3) return xb[f - w.bg_f];
    return xb[3 + f - w.ba_f];
}

// Cost + residuals/Jacobians + normal-equation statistics at (xp, xl, xv, xb) in one walk:
// BAFactor::Evaluate per observation lane (Factors.cpp:327-542) with Huber/Corrector scaling,
// the scaled r/J stored for the step (SoA), per-landmark V = Jl^T Jl and g_l = Jl^T r, per-pose
// U = Jp^T Jp and g_p = Jp^T r, then the IMU factors and the f-space gradient (lin_tail).
// Returns the total cost of the ACTIVE residual blocks; sets sh.st.fail on a PnP evaluation failure.
__device__ __forceinline__ double eval_lin(BaShared& sh, const WinCtx& c, const double* xp, const double* xl, const double* xv,
                           const double* xb, bool first) {
    const BaWin& w = *c.w;
    const int N = w.N, K = w.K, L = w.L;
    pose_cache(sh, c, xp);
    __syncthreads();
    // R_bw at this linearisation point for the Schur / back-substitution walks (later barriers order it)
    for (int e = threadIdx.x; e < 9 * K; e += BA_THREADS) sh.Rlin[e / 9][e % 9] = sh.pc[e / 9][12 + e % 9];
    const Walk g = walk_geom(K);
    const int pf = g.on ? sh.posef[g.kf] : -1;
    const int* lk = reinterpret_cast<const int*>(c.ws + c.L.lk);
    double* r0 = c.ws + c.L.r;
    double* ja = c.ws + c.L.jp;          // A [6][N]
    double* pbw = c.ws + c.L.jp + 6 * (int64_t)N;  // Pb [3][N]
    double* V = c.ws + c.L.V;
    double* gl = c.ws + c.L.gl;
    double* sl = c.ws + c.L.s_l;
    double acc[27];
#pragma unroll
    for (int i = 0; i < 27; ++i) acc[i] = 0.0;
    double cost = 0.0, gm = 0.0;
    int fail = 0;
    // software pipeline: observation index two chunks ahead, its inputs one chunk ahead
    struct EvD { double P[3]; float u, v; int o, lv, out; };
    auto ld_o = [&](int l0n) -> int {
        const int l = l0n + g.jf;
        return (g.on && l < L) ? lk[16 * l + g.kf] : -1;
    };
    auto ld_ev = [&](int l0n, int o, EvD& d) {
        d.o = o;
        if (o >= 0) {
            const int l = l0n + g.jf;
            d.lv = c.lm_var[l];
            d.out = c.outlier[o];
            d.u = c.obs_uv[2 * o];
            d.v = c.obs_uv[2 * o + 1];
            d.P[0] = xl[3 * l]; d.P[1] = xl[3 * l + 1]; d.P[2] = xl[3 * l + 2];
        }
    };
    EvD cur;
    int o_nn = ld_o(g.LC);
    ld_ev(0, ld_o(0), cur);
    for (int l0 = 0, ci = 0; l0 < L; l0 += g.LC, ++ci) {
        EvD nxt;
        nxt.o = -1;
        int o_n2 = -1;
        if (l0 + g.LC < L) {
            ld_ev(l0 + g.LC, o_nn, nxt);
            o_n2 = ld_o(l0 + 2 * g.LC);
        }
        const int o = cur.o;
        double v9[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) v9[i] = 0.0;
        if (o >= 0) {
            const bool lv = cur.lv != 0;
            if (pf >= 0 || lv) {
                double Pw[3] = {cur.P[0], cur.P[1], cur.P[2]};
                double r[2], Aj[6], Pb[3];
                bool jz;
                const int f = factor_eval_ap(sh.pc[g.kf], sh.Rcb_raw[g.kf], Pw, (double)cur.u, (double)cur.v, w.cols,
                                             w.rows, w.Lw, cur.out != 0, w.is_pnp, r, Aj, Pb, jz);
                if (f) {
                    fail = 1;
                } else {
                    double cst, sc;
                    huber(w.huber, r[0] * r[0] + r[1] * r[1], cst, sc);
                    cost += cst;
                    const double ra = r[0] * sc, rb = r[1] * sc;
                    r0[o] = ra;
                    r0[N + o] = rb;
#pragma unroll
                    for (int i = 0; i < 6; ++i) {
                        Aj[i] = jz ? 0.0 : Aj[i] * sc;
                        ja[(int64_t)i * N + o] = Aj[i];
                    }
#pragma unroll
                    for (int i = 0; i < 3; ++i) {
                        Pb[i] = jz ? 0.0 : Pb[i];
                        pbw[(int64_t)i * N + o] = Pb[i];
                    }
                    double Jp[12], Jl[6];
                    jac_from_ap(Aj, Pb, sh.pc[g.kf] + 12, Jp, Jl);
                    double a[6], b[6], la[3], lb[3];
#pragma unroll
                    for (int i = 0; i < 6; ++i) { a[i] = Jp[i]; b[i] = Jp[6 + i]; }
#pragma unroll
                    for (int i = 0; i < 3; ++i) { la[i] = Jl[i]; lb[i] = Jl[3 + i]; }
                    if (pf >= 0) {
                        int idx = 0;
#pragma unroll
                        for (int i = 0; i < 6; ++i)
#pragma unroll
                            for (int j = i; j < 6; ++j) acc[idx++] += a[i] * a[j] + b[i] * b[j];
#pragma unroll
                        for (int i = 0; i < 6; ++i) acc[21 + i] += a[i] * ra + b[i] * rb;
                    }
                    if (lv) {
                        v9[0] = la[0] * la[0] + lb[0] * lb[0];
                        v9[1] = la[0] * la[1] + lb[0] * lb[1];
                        v9[2] = la[0] * la[2] + lb[0] * lb[2];
                        v9[3] = la[1] * la[1] + lb[1] * lb[1];
                        v9[4] = la[1] * la[2] + lb[1] * lb[2];
                        v9[5] = la[2] * la[2] + lb[2] * lb[2];
                        v9[6] = la[0] * ra + lb[0] * rb;
                        v9[7] = la[1] * ra + lb[1] * rb;
                        v9[8] = la[2] * ra + lb[2] * rb;
                    }
                }
            }
        }
        // landmark sums over the slot's K lanes (double-buffered: one barrier per chunk)
        double* rb_ = sh.S + (ci & 1) * 9 * BA_THREADS;
#pragma unroll
        for (int i = 0; i < 9; ++i) rb_[i * BA_THREADS + threadIdx.x] = v9[i];
        if (kProfWalk) prof_mark(sh, PF_EV_F);
        __syncthreads();
        gm = lm_sums9(rb_, l0, g, K, L, c.lm_var, xl, V, gl, sl, first, gm);
        if (kProfWalk) prof_mark(sh, PF_EV_L);
        cur = nxt;
        o_nn = o_n2;
    }
    prof_mark(sh, PF_EVAL_J);
    // pose sums: lanes of one keyframe combined in slot order
    __syncthreads();
    double* pr = sh.S;
#pragma unroll
    for (int i = 0; i < 27; ++i) pr[i * BA_THREADS + threadIdx.x] = acc[i];
    cost += imu_factors(sh, c, xv, xb, true);
    __syncthreads();
    prof_mark(sh, PF_IMU);
    for (int e = threadIdx.x; e < 27 * K; e += BA_THREADS) {
        const int k = e / 27, i = e - 27 * k;
        if (sh.posef[k] < 0) continue;
        double s = 0.0;
#pragma unroll 8
        for (int j = 0; j < g.LC; ++j) s += pr[i * BA_THREADS + j * K + k];
        sh.U[k][i] = s;
    }
    const double total = block_sum(cost, sh.red);
    const double anyfail = block_max((double)fail, sh.redm);
    if (threadIdx.x == 0 && anyfail > 0.0) sh.st.fail = 1;
    __syncthreads();
    lin_tail(sh, c, first, gm, xp, xv, xb);
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

// After eval_lin: IMU normal equations (imu-space H, g), f-space gradient, column norms (Jacobi
// scaling at iteration 0) and the gradient max-norm (gm = landmark part from the walk).
__device__ __forceinline__ void lin_tail(BaShared& sh, const WinCtx& c, bool first, double gm, const double* xp,
                                         const double* xv, const double* xb) {
    const BaWin& w = *c.w;
    const int K = w.K;
    // IMU: per-factor residual/J already in LDS; assemble imu-space H (global) and g.  Factors are
    // added one after another (fixed order); inside a factor the 12 columns map to distinct entries.
    if (w.is_vi) {
        // imu-space H and g accumulated in LDS (the S area is free until compute_step), factors
        // added in order (one barrier per factor; inside a factor the 12 columns map to distinct
        // entries), then written to the workspace once
        const int ni = w.ni;
        double* Hs = sh.S;
        double* gs = sh.S + NI_MAX * NI_MAX;
        for (int e = threadIdx.x; e < ni * ni + ni; e += BA_THREADS) Hs[e < ni * ni ? e : NI_MAX * NI_MAX + e - ni * ni] = 0.0;
        __syncthreads();
        for (int k = 1; k < K; ++k) {
            if (!sh.pvalid[k]) continue;
            const int e = threadIdx.x;
            if (e < 144) {
                const int cp = e / 12, cq = e - 12 * (e / 12);
                const int p = sh.icol[k][cp], q = sh.icol[k][cq];
                if (p >= 0 && q >= 0) {
                    double h = 0.0;
#pragma unroll
                    for (int i = 0; i < 9; ++i) h += sh.imu_J[k][12 * i + cp] * sh.imu_J[k][12 * i + cq];
                    Hs[p * ni + q] += h;
                }
            } else if (e < 156) {
                const int cp = e - 144;
                const int p = sh.icol[k][cp];
                if (p >= 0) {
                    double g = 0.0;
#pragma unroll
                    for (int i = 0; i < 9; ++i) g += sh.imu_J[k][12 * i + cp] * sh.imu_r[k][i];
                    gs[p] += g;
                }
            }
            __syncthreads();
        }
        for (int e = threadIdx.x; e < ni * ni; e += BA_THREADS) c.Himu[e] = Hs[e];
        for (int e = threadIdx.x; e < ni; e += BA_THREADS) c.gimu[e] = gs[e];
    }
    __syncthreads();
    prof_mark(sh, PF_IMUH);
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
            g = sh.S[NI_MAX * NI_MAX + p];   // the LDS copies of gimu / Himu (lin_tail above)
            cs = sh.S[p * w.ni + p];
        }
        sh.g_f[f] = g;
        sh.colsq_f[f] = cs;
        gm = fmax(gm, grad_term(f_param_value(w, f, xp, xv, xb), g));
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
__device__ __forceinline__ void assemble_S(BaShared& sh, const WinCtx& c) {
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

// Schur GEMM (schur_eliminator_impl.h:179-377): with V~_l = L_l L_l^T (L_l^-1 kept per landmark),
// S_pp -= Z Z^T and b_p -= Z h over landmark chunks, where Z = W~ L^-T (the pose x landmark block,
// 6x3 per observation) and h = L^-1 g~_l.  One k-major LDS panel Zt (k = 3*landmark slot + comp)
// feeds both MFMA operands: a step reads T fragments and issues all T(T+1)/2 lower-triangle tile
// products (v_mfma_f64_16x16x4_f64).  The k-steps of a chunk are split over the waves (every wave
// owns every tile: no per-tile branches, balanced), partial tiles are combined wave after wave
// into S at the end (fixed order).  Two panel buffers: while the matrix cores run chunk c, the
// fill lanes (landmark slot, keyframe) write chunk c+1 from registers whose global loads were
// issued one chunk earlier; one barrier per chunk.  Bitwise reproducible.
using d4 = __attribute__((ext_vector_type(4))) double;

constexpr int BA_PANEL = BA_NF_MAX * (BA_NF_MAX + 1) + BA_STAGE;  // S followed by stage
__host__ __device__ constexpr int schur_ks(int T) { return (T & 1) ? 16 * T : 16 * T + 16; }
__host__ __device__ constexpr int schur_kc(int LC) { return (3 * LC + 3) & ~3; }
__host__ __device__ constexpr int schur_lc(int T) {
    int lc = 1;
    while (2 * schur_kc(lc + 1) * schur_ks(T) <= BA_PANEL && 2 * schur_kc(lc + 1) <= BA_GCOL) ++lc;
    return lc;
}

template <int TM>
__device__ __forceinline__ void schur_gemm(BaShared& sh, const WinCtx& c) {
    const BaWin& w = *c.w;
    const int N = w.N, L = w.L, K = w.K, np = w.np;
    constexpr int T = TM;               // pose-row tiles
    constexpr int NT = T * (T + 1) / 2;
    constexpr int G = T >= 5 ? 2 : 1;   // wave groups: each owns a contiguous range of the NT tiles
    constexpr int H = (NT + G - 1) / G; // tiles per group (accumulator registers: 8 per tile)
    constexpr int KS = schur_ks(T);     // k-row stride (doubles): a fragment's 4 k-rows hit both bank halves
    constexpr int LCMAX = schur_lc(T);
    constexpr int NW = BA_THREADS / 64;
    const int LC = min(LCMAX, BA_THREADS / K);  // landmarks per chunk: one fill lane per (landmark, keyframe)
    const int KC = schur_kc(LC);
    const int wid = wave_id(), lane = threadIdx.x & 63;
    const int r16 = lane & 15, kk = lane >> 4;
    const double* ja = c.ws + c.L.jp;                    // A [6][N]
    const double* pbw = c.ws + c.L.jp + 6 * (int64_t)N;  // Pb [3][N]
    const double* Li = c.ws + c.L.Vi;   // L^-1 of V~ per landmark: i00 i10 i11 i20 i21 i22
    const double* gl = c.ws + c.L.gl;
    const double* sl = c.ws + c.L.s_l;
    const int* lk = reinterpret_cast<const int*>(c.ws + c.L.lk);
    d4 acc[H];
#pragma unroll
    for (int t = 0; t < H; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
    constexpr int WPG = (BA_THREADS / 64) / G;  // waves per group: they split the k-steps
    const int grp = wave_id() / WPG, mem = wave_id() - grp * WPG;
    double bacc[T];
#pragma unroll
    for (int r = 0; r < T; ++r) bacc[r] = 0.0;

    const int jf = threadIdx.x / K, kf = threadIdx.x - jf * K;
    const int pf = jf < LC ? sh.posef[kf] : -1;
    // prefetch registers (one chunk ahead); a loaded value is consumed only where it is used
    int o_nx = -1, v_nx = 0;
    double aj[6], pbv[3], sv[3], li[6];
    double hg[3], hs[3], hl[6];
    double rbw[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) rbw[i] = sh.Rlin[kf < BA_KMAX ? kf : 0][i];
    int hv = 0;
    auto load_obs = [&](int l0n, int& o, int& v) {
        const int l = l0n + jf;
        o = -1;
        v = 0;
        if (pf >= 0 && l < L) { o = lk[16 * l + kf]; v = c.lm_var[l]; }  // independent loads
    };
    auto load_data = [&](int l0n, int o) {
        const int l = l0n + jf;
        if (o >= 0) {
#pragma unroll
            for (int i = 0; i < 6; ++i) aj[i] = ja[(int64_t)i * N + o];
#pragma unroll
            for (int i = 0; i < 3; ++i) pbv[i] = pbw[(int64_t)i * N + o];
#pragma unroll
            for (int i = 0; i < 3; ++i) sv[i] = sl[(int64_t)i * L + l];
#pragma unroll
            for (int i = 0; i < 6; ++i) li[i] = Li[(int64_t)i * L + l];
        }
        hv = 0;
        const int lg = l0n + (int)threadIdx.x;
        if ((int)threadIdx.x < LC && lg < L) {
            hv = c.lm_var[lg];
#pragma unroll
            for (int i = 0; i < 3; ++i) { hg[i] = gl[(int64_t)i * L + lg]; hs[i] = sl[(int64_t)i * L + lg]; }
#pragma unroll
            for (int i = 0; i < 6; ++i) hl[i] = Li[(int64_t)i * L + lg];
        }
    };
    auto fill = [&](int buf, int o) {
        double* Zt = sh.S + buf * KC * KS;
        if (pf >= 0) {
            double Z[6][3];
            if (o >= 0) {
                double pj[12], lj[6];
                jac_from_ap(aj, pbv, rbw, pj, lj);
                const double b0 = lj[0] * sv[0], b1 = lj[1] * sv[1], b2 = lj[2] * sv[2];
                const double d0 = lj[3] * sv[0], d1 = lj[4] * sv[1], d2 = lj[5] * sv[2];
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    const double sp = sh.s_f[pf + i];
                    const double a = pj[i] * sp, e = pj[6 + i] * sp;
                    const double W0 = a * b0 + e * d0, W1 = a * b1 + e * d1, W2 = a * b2 + e * d2;
                    Z[i][0] = W0 * li[0];
                    Z[i][1] = W0 * li[1] + W1 * li[2];
                    Z[i][2] = W0 * li[3] + W1 * li[4] + W2 * li[5];
                }
            } else {
#pragma unroll
                for (int i = 0; i < 6; ++i)
#pragma unroll
                    for (int cc = 0; cc < 3; ++cc) Z[i][cc] = 0.0;
            }
#pragma unroll
            for (int cc = 0; cc < 3; ++cc)
#pragma unroll
                for (int i = 0; i < 6; ++i) Zt[(3 * jf + cc) * KS + pf + i] = Z[i][cc];
        }
        if ((int)threadIdx.x < LC) {
            double* G = sh.gcol + buf * KC;
            double h0 = 0.0, h1 = 0.0, h2 = 0.0;
            if (hv) {
                const double g0 = hg[0] * hs[0], g1 = hg[1] * hs[1], g2 = hg[2] * hs[2];
                h0 = hl[0] * g0;
                h1 = hl[1] * g0 + hl[2] * g1;
                h2 = hl[3] * g0 + hl[4] * g1 + hl[5] * g2;
            }
            G[3 * threadIdx.x] = h0;
            G[3 * threadIdx.x + 1] = h1;
            G[3 * threadIdx.x + 2] = h2;
        }
    };
    // both panels zero: rows of constant poses, padding rows and padding k-rows stay zero
    for (int e = threadIdx.x; e < 2 * KC * KS; e += BA_THREADS) sh.S[e] = 0.0;
    for (int e = threadIdx.x; e < 2 * KC; e += BA_THREADS) sh.gcol[e] = 0.0;
    {
        int o0, v0;
        load_obs(0, o0, v0);
        load_data(0, v0 ? o0 : -1);
        __syncthreads();
        fill(0, v0 ? o0 : -1);
    }
    if (LC < L) {
        load_obs(LC, o_nx, v_nx);
        load_data(LC, v_nx ? o_nx : -1);
    }
    __syncthreads();
    prof_mark(sh, PF_FILL);
    for (int l0 = 0, ci = 0; l0 < L; l0 += LC, ++ci) {
        const int buf = ci & 1;
        const int l1 = min(l0 + LC, L);
        // ---- matrix cores: this wave's k-steps of chunk ci
        {
            const double* Zt = sh.S + buf * KC * KS;
            const double* Gc = sh.gcol + buf * KC;
            const int nsteps = (3 * (l1 - l0) + 3) >> 2;
            for (int st = mem; st < nsteps; st += WPG) {
                const int kr = (4 * st + kk) * KS;
                double f[T];
#pragma unroll
                for (int r = 0; r < T; ++r) f[r] = Zt[kr + 16 * r + r16];
                if (grp == 0) {
#pragma unroll
                    for (int r = 0, t = 0; r < T; ++r)
#pragma unroll
                        for (int q = 0; q <= r; ++q, ++t)
                            if (t < H) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(f[r], f[q], acc[t], 0, 0, 0);
                    const double g = Gc[4 * st + kk];
#pragma unroll
                    for (int r = 0; r < T; ++r) bacc[r] += f[r] * g;
                } else {
#pragma unroll
                    for (int r = 0, t = 0; r < T; ++r)
#pragma unroll
                        for (int q = 0; q <= r; ++q, ++t)
                            if (t >= H) acc[t - H] = __builtin_amdgcn_mfma_f64_16x16x4f64(f[r], f[q], acc[t - H], 0, 0, 0);
                }
            }
        }
        prof_mark(sh, PF_GEMM);
        // ---- fill chunk ci+1 into the other buffer, then issue the loads of chunk ci+2
        if (l1 < L) {
            const int o = v_nx ? o_nx : -1;
            fill(buf ^ 1, o);
            if (l1 + LC < L) {
                load_obs(l1 + LC, o_nx, v_nx);
                load_data(l1 + LC, v_nx ? o_nx : -1);
            }
        }
        __syncthreads();
        prof_mark(sh, PF_PFX);
    }
    assemble_S(sh, c);
    // partial tiles and rhs of each wave into S / b, wave after wave (fixed order)
    const int ls = s_ld(w.nf);
#pragma unroll
    for (int r = 0; r < T; ++r) {
        bacc[r] += __shfl_xor(bacc[r], 16, 64);
        bacc[r] += __shfl_xor(bacc[r], 32, 64);
    }
    for (int wv = 0; wv < NW; ++wv) {
        if (wid == wv) {
            auto put = [&](int r, int q, const d4& a) {
                const int col = 16 * q + r16;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = 16 * r + 4 * e + kk;
                    if (row < np && col < np) sh.S[row * ls + col] -= a[e];
                }
            };
            if (grp == 0) {
#pragma unroll
                for (int r = 0, t = 0; r < T; ++r)
#pragma unroll
                    for (int q = 0; q <= r; ++q, ++t)
                        if (t < H) put(r, q, acc[t]);
            } else {
#pragma unroll
                for (int r = 0, t = 0; r < T; ++r)
#pragma unroll
                    for (int q = 0; q <= r; ++q, ++t)
                        if (t >= H) put(r, q, acc[t - H]);
            }
#pragma unroll
            for (int r = 0; r < T; ++r) {
                const int row = 16 * r + r16;
                if (kk == 0 && row < np) sh.b[row] -= bacc[r];
            }
        }
        __syncthreads();
    }
    prof_mark(sh, PF_ASM);
}

// Cholesky of S (nf x nf in LDS, padded to nb = ceil(nf/16) 16x16 tiles with an identity tail,
// row stride s_ld(nf)) then solve S y = b (y overwrites b).  Blocked right-looking:
//   (A) wave 0 factors the diagonal tile in registers (lane i = row i; pivots and column entries
//       broadcast with v_readlane; 1/sqrt by v_rsq_f64 + two Newton steps), writes the tile's L to
//       LDS and forms the triangular inverse from LDS broadcast reads; Linv_J^T goes to the stage area;
//   (B) panel tiles L_IJ = S_IJ Linv_J^T on v_mfma_f64_16x16x4_f64, one tile per wave at a time;
//   (C) trailing lower tiles S_IK -= L_IJ L_KJ^T on the matrix cores.
// chol16_wave (chol_dev.h) is the wave-level tile factor.  Three workgroup barriers per tile column.  The two triangular solves walk the tile columns with
// one wave (lanes = 16 rows x 4 column groups; the tile's right-hand side is broadcast through LDS).
// Fixed operation order: bitwise reproducible.  (tools/probe/chol_probe.hip times the variants.)
// Returns false (uniformly) when a pivot is not positive (S not positive definite).
struct NoStamp {
    __device__ void operator()(int) const {}
};
// stamp(slot): optional diagnostic marks (diagonal tiles 8, panels 9, trailing updates 10, forward 11,
// backward 12)
template <typename Stamp = NoStamp>
__device__ __forceinline__ bool cholesky_solve(BaShared& sh, int nf, Stamp stamp = Stamp()) {
    double* S = sh.S;
    double* LB = sh.stage;  // [nb][16 m][16 c] = Linv_J[c][m]
    double* LT = sh.stage + 256 * ((BA_NF_MAX + 15) >> 4);  // [16 m][16 q] = L_JJ[q][m]; then 16 rhs
    double* TB = LT + 256;
    const int ls = s_ld(nf), nb = (nf + 15) >> 4;
    constexpr int NW = BA_THREADS / 64;
    const int wid = wave_id(), lane = threadIdx.x & 63;
    const int r16 = lane & 15, kk = lane >> 4;
    for (int J = 0; J < nb; ++J) {
        const int c0 = 16 * J;
        // (A) diagonal tile
        if (wid == 0) {
            const int bad = chol16_wave<false>(S + c0 * ls + c0, ls, LB + 256 * J, LT, lane);
            if (lane == 0) sh.chol_bad = bad;
        }
        __syncthreads();
        stamp(8);
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
        stamp(9);
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
        stamp(10);
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
            if (kk == 0) TB[r16] = t;
            wave_lds_sync();
            double v = 0.0;
#pragma unroll
            for (int q = 0; q < 4; ++q) v += lb[16 * (kk + 4 * q) + r16] * TB[kk + 4 * q];
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            if (kk == 0) y[16 * J + r16] = v;
            wave_lds_sync();
        }
        stamp(11);
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
            if (kk == 0) TB[r16] = t;
            wave_lds_sync();
            double v = 0.0;
#pragma unroll
            for (int q = 0; q < 4; ++q) v += lb[16 * r16 + kk + 4 * q] * TB[kk + 4 * q];
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            if (kk == 0) y[16 * J + r16] = v;
            wave_lds_sync();
        }
        stamp(12);
    }
    __syncthreads();
    return true;
}

// Phase-route variant of cholesky_solve for nf % 16 != 0 (ph_solve): the right-hand side is carried
// as row nf of S (columns < nf; S[nf][nf] = kRhsPivot, the padding rows below it identity), so the
// factorisation itself produces y = L^-1 b as L[nf][0..nf) (the forward substitution runs in the
// panels / trailing updates / diagonal tiles; the diagonal tiles are overwritten with their L).  One-step look-ahead: after the panel of column J,
// wave 0 updates the next diagonal tile and factors it while the other waves apply the rest of
// column J's trailing update (two workgroup barriers per tile column).  Then the backward solve as
// in cholesky_solve.  Returns false (uniformly) when a pivot of rows < nf is not positive.
constexpr double kRhsPivot = 1e300;
template <typename Stamp = NoStamp>
__device__ __forceinline__ bool cholesky_solve_rhs(BaShared& sh, int nf, Stamp stamp = Stamp()) {
    double* S = sh.S;
    double* LB = sh.stage;  // [nb][16 m][16 c] = Linv_J[c][m]
    double* LT = sh.stage + 256 * ((BA_NF_MAX + 15) >> 4);
    double* TB = LT + 256;
    const int ls = s_ld(nf), nb = (nf + 15) >> 4;
    constexpr int NW = BA_THREADS / 64;
    const int wid = wave_id(), lane = threadIdx.x & 63;
    const int r16 = lane & 15, kk = lane >> 4;
    // trailing update of the lower tile (I, K) by column J
    auto trail = [&](int I, int Kt, int J) {
        const int c0 = 16 * J;
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
    };
    if (wid == 0) {
        const int bad = chol16_wave<true>(S, ls, LB, LT, lane, min(16, nf));
        if (lane == 0) sh.chol_bad = bad;
    }
    __syncthreads();
    stamp(8);
    if (sh.chol_bad) return false;
    for (int J = 0; J < nb; ++J) {
        const int c0 = 16 * J;
        // panel: L_IJ = S_IJ Linv_J^T
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
        stamp(9);
        if (J + 1 == nb) break;
        if (wid == 0) {
            // look-ahead: the next diagonal tile, updated by column J, then factored
            trail(J + 1, J + 1, J);
            wave_lds_sync();
            const int bad = chol16_wave<true>(S + (c0 + 16) * ls + c0 + 16, ls, LB + 256 * (J + 1), LT, lane,
                                               min(16, nf - c0 - 16));
            if (lane == 0) sh.chol_bad = bad;
        } else {
            // the rest of column J's trailing update: lower tiles (I, K), J < K <= I < nb, except (J+1, J+1)
            const int m = nb - J - 1, nt = m * (m + 1) / 2;
            for (int t = wid; t < nt; t += NW - 1) {
                int I = 0, tt = t;
                while (tt > I) { tt -= I + 1; ++I; }
                if (I == 0) continue;  // tile (J+1, J+1): wave 0
                trail(I + J + 1, tt + J + 1, J);
            }
        }
        __syncthreads();
        stamp(10);
        if (sh.chol_bad) return false;
    }
    // y = L^-1 b is row nf of L; the backward solve x_J = Linv_J^T (y_J - sum_{K>J} L_KJ^T x_K) by wave 0
    if (wid == 0) {
        double* y = sh.b;
        for (int f = lane; f < 16 * nb; f += 64) y[f] = f < nf ? S[nf * ls + f] : 0.0;
        wave_lds_sync();
        stamp(11);
        for (int J = nb - 1; J >= 0; --J) {
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
            if (kk == 0) TB[r16] = t;
            wave_lds_sync();
            double v = 0.0;
#pragma unroll
            for (int q = 0; q < 4; ++q) v += lb[16 * r16 + kk + 4 * q] * TB[kk + 4 * q];
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            if (kk == 0) y[16 * J + r16] = v;
            wave_lds_sync();
        }
        stamp(12);
    }
    __syncthreads();
    return true;
}

// One LM step computation (ComputeTrustRegionStep): returns validity uniformly via sh.st.valid.
__device__ __forceinline__ void compute_step(BaShared& sh, const WinCtx& c) {
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
        Vi[l] = i00;   // L^-1 (lower): V~^-1 = L^-T L^-1 is applied factor by factor
        Vi[(int64_t)L + l] = i10;
        Vi[2 * (int64_t)L + l] = i11;
        Vi[3 * (int64_t)L + l] = i20;
        Vi[4 * (int64_t)L + l] = i21;
        Vi[5 * (int64_t)L + l] = i22;
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
    // (5) back-substitution for the points, y_l = V~^-1 (g~_l - W~^T y_p), in one walk with the
    // observation part of the model change -(J delta)^T (r + J delta / 2) (trust_region_minimizer.cc
    // :424-439) and the landmark candidates: the Jacobians are read once, coalesced.
    for (int f = threadIdx.x; f < nf; f += BA_THREADS) sh.D_f[f] = -sh.b[f] * sh.s_f[f];  // delta_f
    __syncthreads();
    const int K = w.K;
    double fin = 0.0, mc = 0.0, sn = 0.0, xn = 0.0;
    double ccost = 0.0;  // cost at the candidate (TrustRegionMinimizer evaluates it next; fused here)
    int cfail = 0;
    double* ws = c.ws;
    double* xp = ws + c.L.x_pose; double* cp_ = ws + c.L.c_pose;
    double* xv = ws + c.L.x_vel;  double* cv = ws + c.L.c_vel;
    double* xb = ws + c.L.x_bias; double* cb = ws + c.L.c_bias;
    for (int e = threadIdx.x; e < 6 * K; e += BA_THREADS) {
        int k = e / 6, i = e % 6;
        int pfk = w.pose_f[k];
        double x = xp[e];
        double cnd = pfk >= 0 ? x + sh.D_f[pfk + i] : x;
        cp_[e] = cnd;
        if (pfk >= 0) { double d = x - cnd; sn += d * d; xn += cnd * cnd; }
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
            bool a = e < 3 ? w.bg_f >= 0 : w.ba_f >= 0;
            double x = xb[e];
            double cnd = a ? x + sh.D_f[f] : x;
            cb[e] = cnd;
            if (a) { double d = x - cnd; sn += d * d; xn += cnd * cnd; }
        }
    }
    __syncthreads();
    pose_cache(sh, c, cp_);  // sh.pc now holds the candidate poses (the step uses sh.Rlin)
    __syncthreads();
    const Walk g = walk_geom(K);
    const int pf = g.on ? sh.posef[g.kf] : -1;
    const int* lk = reinterpret_cast<const int*>(c.ws + c.L.lk);
    const double* r0 = c.ws + c.L.r;
    const double* ja = c.ws + c.L.jp;                    // A [6][N]
    const double* pbw = c.ws + c.L.jp + 6 * (int64_t)N;  // Pb [3][N]
    const double* xl = c.ws + c.L.x_lm;
    double* cl = c.ws + c.L.c_lm;
    double rbw[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) rbw[i] = sh.Rlin[g.kf < BA_KMAX ? g.kf : 0][i];
    double* red = sh.S;                    // [3][BA_THREADS] per-lane W^T-terms
    double* dls = sh.S + 3 * BA_THREADS;   // [LC][3] landmark steps of the chunk
    double* cps = sh.S + 6 * BA_THREADS;   // [LC][3] landmark candidates of the chunk
    // software pipeline: observation index two chunks ahead, observation data one chunk ahead
    struct ObsD { double a6[6], pb[3], ra, rb; float u, v; int o, lv, out; };
    struct LmD { double sv[3], gv[3], vi[6], x[3]; int lv; };
    auto ld_o = [&](int l0n) -> int {
        const int l = l0n + g.jf;
        return (g.on && l < L) ? lk[16 * l + g.kf] : -1;
    };
    auto ld_obs = [&](int l0n, int o, ObsD& d) {
        d.o = o;
        d.lv = 0;
        if (o >= 0) {
            d.lv = c.lm_var[l0n + g.jf];
#pragma unroll
            for (int i = 0; i < 6; ++i) d.a6[i] = ja[(int64_t)i * N + o];
#pragma unroll
            for (int i = 0; i < 3; ++i) d.pb[i] = pbw[(int64_t)i * N + o];
            d.ra = r0[o];
            d.rb = r0[N + o];
            d.u = c.obs_uv[2 * o];
            d.v = c.obs_uv[2 * o + 1];
            d.out = c.outlier[o];
        }
    };
    auto ld_lm = [&](int l0n, LmD& d) {
        const int lj = l0n + threadIdx.x;
        d.lv = 0;
        if ((int)threadIdx.x < g.LC && lj < L) {
            d.lv = c.lm_var[lj];
#pragma unroll
            for (int cc = 0; cc < 3; ++cc) {
                d.sv[cc] = sl[(int64_t)cc * L + lj];
                d.gv[cc] = gl[(int64_t)cc * L + lj];
                d.x[cc] = xl[3 * lj + cc];
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) d.vi[i] = Vi[(int64_t)i * L + lj];
        }
    };
    ObsD cur;
    int o_nn = ld_o(g.LC);
    ld_obs(0, ld_o(0), cur);
    for (int l0 = 0; l0 < L; l0 += g.LC) {
        // landmark-lane data of this chunk: issued here, consumed after the first barrier (a prefetch
        // one chunk ahead would live across the candidate evaluation and spill)
        LmD lcur;
        ld_lm(l0, lcur);
        ObsD nxt;
        nxt.o = -1; nxt.lv = 0;
        int o_n2 = -1;
        if (l0 + g.LC < L) {
            ld_obs(l0 + g.LC, o_nn, nxt);
            o_n2 = ld_o(l0 + 2 * g.LC);
        }
        const bool lv = cur.o >= 0 && cur.lv;
        const bool act = cur.o >= 0 && (pf >= 0 || cur.lv);
        double e0 = 0.0, e1 = 0.0;
        double j6[6], p12[12];
        jac_from_ap(cur.a6, cur.pb, rbw, p12, j6);
        if (act && pf >= 0) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double d = sh.D_f[pf + i];
                e0 += p12[i] * d;
                e1 += p12[6 + i] * d;
            }
        }
        const bool contrib = lv && pf >= 0;
#pragma unroll
        for (int cc = 0; cc < 3; ++cc)
            red[cc * BA_THREADS + threadIdx.x] = contrib ? j6[cc] * e0 + j6[3 + cc] * e1 : 0.0;
        __syncthreads();
        if (kProfWalk) prof_mark(sh, PF_BS_J);
        if ((int)threadIdx.x < g.LC) {
            const int lj = l0 + threadIdx.x;
            if (lj < L) {
                double d[3] = {0.0, 0.0, 0.0};
                if (lcur.lv) {
                    double rhs[3];
#pragma unroll
                    for (int cc = 0; cc < 3; ++cc) {
                        double t = 0.0;
#pragma unroll
                        for (int kf = 0; kf < BA_KMAX; ++kf)
                            if (kf < K) t += red[cc * BA_THREADS + threadIdx.x * K + kf];
                        rhs[cc] = lcur.gv[cc] * lcur.sv[cc] + lcur.sv[cc] * t;
                    }
                    const double* li = lcur.vi;  // y = L^-T (L^-1 rhs)
                    const double t0 = li[0] * rhs[0];
                    const double t1 = li[1] * rhs[0] + li[2] * rhs[1];
                    const double t2 = li[3] * rhs[0] + li[4] * rhs[1] + li[5] * rhs[2];
                    const double y0 = li[0] * t0 + li[1] * t1 + li[3] * t2;
                    const double y1 = li[2] * t1 + li[4] * t2;
                    const double y2 = li[5] * t2;
                    yl[lj] = y0;
                    yl[(int64_t)L + lj] = y1;
                    yl[2 * (int64_t)L + lj] = y2;
                    if (!isfinite(y0) || !isfinite(y1) || !isfinite(y2)) fin = 1.0;
                    d[0] = -y0 * lcur.sv[0];
                    d[1] = -y1 * lcur.sv[1];
                    d[2] = -y2 * lcur.sv[2];
                }
#pragma unroll
                for (int cc = 0; cc < 3; ++cc) {
                    const double x = lcur.x[cc];
                    const double cnd = lcur.lv ? x + d[cc] : x;
                    cl[3 * lj + cc] = cnd;
                    if (lcur.lv) {
                        const double dd = x - cnd;
                        sn += dd * dd;
                        xn += cnd * cnd;
                    }
                    dls[3 * threadIdx.x + cc] = d[cc];
                    cps[3 * threadIdx.x + cc] = cnd;
                }
            }
        }
        __syncthreads();
        if (kProfWalk) prof_mark(sh, PF_BS_L);
        if (act) {
            double m0 = e0, m1 = e1;
            if (lv) {
#pragma unroll
                for (int cc = 0; cc < 3; ++cc) {
                    const double d = dls[3 * g.jf + cc];
                    m0 += j6[cc] * d;
                    m1 += j6[3 + cc] * d;
                }
            }
            mc -= m0 * (cur.ra + m0 / 2.0) + m1 * (cur.rb + m1 / 2.0);
            // the residual block at the candidate (point + pose of this lane)
            double Pc[3] = {cps[3 * g.jf], cps[3 * g.jf + 1], cps[3 * g.jf + 2]};
            double r[2], Jp[12], Jl[6];
            bool jz;
            if (factor_eval(sh.pc[g.kf], sh.Rcb_raw[g.kf], Pc, (double)cur.u, (double)cur.v, w.cols, w.rows, w.Lw,
                            cur.out != 0, w.is_pnp, false, r, Jp, Jl, jz)) {
                cfail = 1;
            } else {
                double cst, sc;
                huber(w.huber, r[0] * r[0] + r[1] * r[1], cst, sc);
                ccost += cst;
            }
        }
        if (kProfWalk) prof_mark(sh, PF_BS_C);
        cur = nxt;
        o_nn = o_n2;
    }
    for (int f = threadIdx.x; f < nf; f += BA_THREADS)
        if (!isfinite(sh.b[f])) fin = 1.0;
    prof_mark(sh, PF_BACKSUB);
    // IMU part of the model change
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
    ccost += imu_factors(sh, c, cv, cb, false);  // IMU factors at the candidate
    const double nonfinite = block_max(fin, sh.redm);
    const double mct = block_sum(mc, sh.red);
    const double snt = block_sum(sn, sh.red);
    const double xnt = block_sum(xn, sh.red);
    const double cct = block_sum(ccost, sh.red);
    const double cfl = block_max((double)cfail, sh.redm);
    if (threadIdx.x == 0) {
        sh.st.valid = nonfinite > 0.0 ? 0 : 1;
        sh.st.model_change = mct;
        sh.st.step_norm = sqrt(snt);
        sh.st.cand_x_norm2 = xnt;
        sh.st.fused_cost = cct;
        sh.st.cand_fail = cfl > 0.0 ? 1 : 0;
    }
    __syncthreads();
    prof_mark(sh, PF_CAND);
}

// ---- setup helpers: the lane's loads of several strides are issued before its stores (a loop of
// dependent load -> store pairs costs one memory round trip per stride otherwise)
constexpr int SETUP_U = 4;
// dst[e] = src[e], e < n, by NT threads
template <int NT = BA_THREADS>
__device__ __forceinline__ void copy_strided(double* dst, const double* src, int n) {
    for (int e0 = threadIdx.x; e0 < n; e0 += SETUP_U * NT) {
        double v[SETUP_U];
#pragma unroll
        for (int u = 0; u < SETUP_U; ++u) {
            const int e = e0 + u * NT;
            v[u] = e < n ? src[e] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < SETUP_U; ++u) {
            const int e = e0 + u * NT;
            if (e < n) dst[e] = v[u];
        }
    }
}
// (landmark, keyframe) -> observation table (pairs are unique: host-checked); lk preset to -1
__device__ __forceinline__ void fill_lk(int* lk, const int* obs_lm, const int* obs_kf, int N) {
    for (int o0 = threadIdx.x; o0 < N; o0 += SETUP_U * BA_THREADS) {
        int lm[SETUP_U], kf[SETUP_U];
#pragma unroll
        for (int u = 0; u < SETUP_U; ++u) {
            const int o = o0 + u * BA_THREADS;
            lm[u] = o < N ? obs_lm[o] : 0;
            kf[u] = o < N ? obs_kf[o] : 0;
        }
#pragma unroll
        for (int u = 0; u < SETUP_U; ++u) {
            const int o = o0 + u * BA_THREADS;
            if (o < N) lk[16 * lm[u] + kf[u]] = o;
        }
    }
}
// fixed cost (program.cc:305-390): residual blocks whose pose and point are both constant, in the
// lane's observation order; posef = the window's pose -> f-column table (LDS), pc / rcb its pose cache
template <typename PC, typename RCB>
__device__ __forceinline__ double fixed_cost(const WinCtx& c, const int* posef, const PC& pc, const RCB& rcb) {
    const BaWin& w = *c.w;
    const int N = w.N;
    double fc = 0.0;
    for (int o0 = threadIdx.x; o0 < N; o0 += SETUP_U * BA_THREADS) {
        int kf[SETUP_U], lm[SETUP_U];
#pragma unroll
        for (int u = 0; u < SETUP_U; ++u) {
            const int o = o0 + u * BA_THREADS;
            kf[u] = o < N ? c.obs_kf[o] : 0;
            lm[u] = o < N ? c.obs_lm[o] : 0;
        }
        unsigned fixed = 0;
#pragma unroll
        for (int u = 0; u < SETUP_U; ++u) {
            const int o = o0 + u * BA_THREADS;
            if (o < N && posef[kf[u]] < 0 && !c.lm_var[lm[u]]) fixed |= 1u << u;
        }
        for (int u = 0; u < SETUP_U; ++u) {  // rare: reload the observation
            if (!((fixed >> u) & 1u)) continue;
            const int o = o0 + u * BA_THREADS;
            const int k = c.obs_kf[o], l = c.obs_lm[o];
            double Pw[3] = {c.lm_xyz0[3 * l], c.lm_xyz0[3 * l + 1], c.lm_xyz0[3 * l + 2]};
            double r[2], Jp[12], Jl[6];
            bool jz;
            if (factor_eval(pc[k], rcb[k], Pw, (double)c.obs_uv[2 * o], (double)c.obs_uv[2 * o + 1], w.cols, w.rows,
                            w.Lw, false, w.is_pnp, false, r, Jp, Jl, jz) == 0) {
                double cst, sc;
                huber(w.huber, r[0] * r[0] + r[1] * r[1], cst, sc);
                fc += cst;
            }
        }
    }
    return fc;
}

__device__ __forceinline__ void accept_candidate(BaShared& sh, const WinCtx& c) {
    const BaWin& w = *c.w;
    double* ws = c.ws;
    const int K = w.K, L = w.L;
    copy_strided(ws + c.L.x_pose, ws + c.L.c_pose, 6 * K);
    copy_strided(ws + c.L.x_lm, ws + c.L.c_lm, 3 * L);
    copy_strided(ws + c.L.x_vel, ws + c.L.c_vel, 3 * K);
    copy_strided(ws + c.L.x_bias, ws + c.L.c_bias, 6);
    __syncthreads();
}

// ------------------------------------------------------------------------------------------
// One ceres::Solve from the current workspace point.  Ceres semantics: see trust_region_minimizer.cc.
__device__ __forceinline__ void lm_solve(BaShared& sh, const WinCtx& c) {
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
    double cost = eval_lin(sh, c, xp, xl, xv, xb, true);
    prof_mark(sh, PF_LIN);
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
    if (threadIdx.x == 0) {
        LmState& s = sh.st;
        s.x_cost = cost;
        s.initial_cost = cost + s.fixed_cost;
        s.final_cost = s.initial_cost;
        s.step_eval_current = cost;
        s.step_ok = 1;
        s.iter_cost = cost + s.fixed_cost;
        trace_begin(s);  // IterationZero (:195-229): valid and successful
        s.tr_valid = 1;
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
            trace_push(c, s);
            if (s.iteration >= w.max_iter) { s.termination = VIO_TERM_NO_CONVERGENCE; s.done = 1; }
            else if (!fixed && s.step_ok && s.gmax <= 1e-10) { s.termination = VIO_TERM_CONVERGENCE; s.done = 1; }
            else if (!fixed && s.radius <= 1e-32) { s.termination = VIO_TERM_CONVERGENCE; s.done = 1; }
            if (!s.done) {
                s.iteration++;
                trace_begin(s);
            }
        }
        __syncthreads();
        if (sh.st.done) break;
        prof_mark(sh, PF_CTRL);
        compute_step(sh, c);
        bool valid = sh.st.valid;
        if (valid) {
            if (threadIdx.x == 0) {
                sh.st.tr_model = sh.st.model_change;
                sh.st.valid = sh.st.model_change > 0.0;
            }
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
        // candidate cost: evaluated inside compute_step (same residual blocks, same order of terms per lane)
        double cc = sh.st.fused_cost;
        if (threadIdx.x == 0 && sh.st.cand_fail) sh.st.fail = 1;
        __syncthreads();
        prof_mark(sh, PF_EVAL_C);
        if (threadIdx.x == 0) {
            LmState& s = sh.st;
            s.cand_cost = s.fail ? DBL_MAX : cc;
            s.fail = 0;
            s.tr_valid = 1;
            s.tr_step_norm = s.step_norm;
            s.tr_cost_change = s.x_cost - s.cand_cost;
            if (!fixed && s.step_norm <= 1e-8 * (s.x_norm + 1e-8)) { s.termination = VIO_TERM_CONVERGENCE; s.done = 1; }
            else if (!fixed && fabs(s.x_cost - s.cand_cost) <= 1e-6 * s.x_cost) { s.termination = VIO_TERM_CONVERGENCE; s.done = 1; }
            else {
                double rel = s.cand_cost >= DBL_MAX ? -DBL_MAX : (s.step_eval_current - s.cand_cost) / s.model_change;
                s.rel = rel;
                s.tr_rel = rel;
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
            double nc = eval_lin(sh, c, xp, xl, xv, xb, false);
            prof_mark(sh, PF_LIN);
            if (sh.st.fail) {
                if (threadIdx.x == 0) { sh.st.termination = VIO_TERM_FAILURE; sh.st.done = 1; }
                __syncthreads();
                break;
            }
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
__device__ __forceinline__ void init_params(BaShared& sh, const WinCtx& c, bool poses_only) {
    const BaWin& w = *c.w;
    double* ws = c.ws;
    for (int e = threadIdx.x; e < 6 * w.K; e += BA_THREADS) ws[c.L.x_pose + e] = 0.0;
    if (!poses_only) {
        copy_strided(ws + c.L.x_lm, c.lm_xyz0, 3 * w.L);
        for (int e = threadIdx.x; e < 3 * w.K; e += BA_THREADS) ws[c.L.x_vel + e] = w.is_vi ? c.vel0[e] : 0.0;
        for (int e = threadIdx.x; e < 6; e += BA_THREADS) ws[c.L.x_bias + e] = e < 3 ? w.bg0[e] : w.ba0[e - 3];
    }
    __syncthreads();
}

#ifndef VIO_BA_CLUSTER_TU  // (ba_cluster.hip: the cluster route's kernel alone)
__global__ void __launch_bounds__(BA_THREADS, 1) ba_window_kernel(BaPools P) {
    extern __shared__ __align__(16) unsigned char smem_raw[];
    BaShared& sh = *reinterpret_cast<BaShared*>(smem_raw);
    const BaWin& w = P.win[blockIdx.x];
    if (P.route == 1 && !w.is_pnp) return;  // solved by the phase kernels
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
    c.trace = P.out_trace + w.o_tr;
    const int K = w.K, L = w.L, N = w.N;
    if (threadIdx.x == 0) {
        sh.st.tr_n = 0;
        sh.prof_on = P.prof != nullptr;
        for (int i = 0; i < PF_NSLOT; ++i) sh.prof_acc[i] = 0;
        sh.prof_last = __builtin_amdgcn_s_memtime();
    }
    __syncthreads();

    // ---- setup: projected input rotations (SE3d(T_wb_init), SE3d(T_cb)), raw R_cb, IMU sqrt-info
    {   // three independent serial jobs per keyframe on three different waves (SIMDs): SO3 projection
        // of R_init (wave 0), of R_cb (wave 1), IMU sqrt-information (wave 2); K <= BA_KMAX <= 64
        const int job = threadIdx.x >> 6, k = threadIdx.x & 63;
        if (k < K) {
            const double* pr = c.pose_raw + 24 * k;
            if (job == 0) {
                polar3(pr, sh.pinit[k]);
                for (int i = 0; i < 3; ++i) sh.pinit[k][9 + i] = pr[9 + i];
            } else if (job == 1) {
                polar3(pr + 12, sh.pinit[k] + 12);
                for (int i = 0; i < 3; ++i) sh.pinit[k][21 + i] = pr[21 + i];
                for (int i = 0; i < 9; ++i) sh.Rcb_raw[k][i] = pr[12 + i];
            }
        }
        if (job >= 2 && w.is_vi)  // whole waves 2 and 3, one IMU factor at a time each
            for (int kk = 1 + (job - 2); kk < K; kk += 2)
                if (c.preint_valid[kk]) imu_sqrt_info_wave(c.preint[kk], c.sqi + 81 * kk);
    }
    for (int o = threadIdx.x; o < N; o += BA_THREADS) c.outlier[o] = 0;
    for (int k = threadIdx.x; k < BA_KMAX; k += BA_THREADS) {
        sh.posef[k] = k < K ? w.pose_f[k] : -1;
        sh.pvalid[k] = k < K ? c.preint_valid[k] : 0;
    }
    for (int e = threadIdx.x; e < 12 * BA_KMAX; e += BA_THREADS) {
        const int k = e / 12, cc = e - 12 * k;
        sh.icol[k][cc] = (int8_t)((w.is_vi && k >= 1 && k < K) ? imu_col(w, k, cc) : -1);
    }
    {   // (landmark, keyframe) -> observation table for the Schur fill (pairs are unique: host-checked)
        int* lk = reinterpret_cast<int*>(c.ws + c.L.lk);
        for (int e = threadIdx.x; e < 16 * L; e += BA_THREADS) lk[e] = -1;
        __syncthreads();
        fill_lk(lk, c.obs_lm, c.obs_kf, N);
    }
    init_params(sh, c, false);

    // ---- fixed cost: residual blocks whose parameters are all constant (program.cc:305-390)
    {
        pose_cache(sh, c, c.ws + c.L.x_pose);
        __syncthreads();
        const double fc = fixed_cost(c, sh.posef, sh.pc, sh.Rcb_raw);
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
    if (P.prof && threadIdx.x < PF_NSLOT) P.prof[PF_NSLOT * blockIdx.x + threadIdx.x] = sh.prof_acc[threadIdx.x];
}

// ------------------------------------------------------------------------------------------
// result records (vio_ba_batch_pack): one workgroup per window, every field copied with coalesced
// lanes; outlier flags scattered back to the caller's observation order
__global__ void __launch_bounds__(BA_THREADS) ba_pack_kernel(BaPools P, uint8_t* dst, int64_t rec_bytes) {
    const BaWin& w = P.win[blockIdx.x];
    const int K = w.K, L = w.L, N = w.N;
    const RecLayout R = rec_layout(K, L, N);
    const BaOutLayout OL = ba_out_layout(K, L, N);
    uint8_t* rec = dst + rec_bytes * blockIdx.x;
    const double* out = P.out + w.o_out;
    int32_t* hdr = reinterpret_cast<int32_t*>(rec);
    if (threadIdx.x == 0) { hdr[0] = K; hdr[1] = L; hdr[2] = N; hdr[3] = VIO_BA_RECORD_VERSION; }
    if (threadIdx.x < SI_COUNT) reinterpret_cast<int32_t*>(rec + R.si)[threadIdx.x] = P.out_i32[SI_COUNT * blockIdx.x + threadIdx.x];
    if (threadIdx.x < SD_COUNT)
        reinterpret_cast<double*>(rec + R.sd)[threadIdx.x] = threadIdx.x < 3 ? P.out_sum[SD_COUNT * blockIdx.x + threadIdx.x] : 0.0;
    double* T = reinterpret_cast<double*>(rec + R.T);
    for (int e = threadIdx.x; e < 12 * K; e += BA_THREADS) T[e] = out[OL.T_wb + e];
    double* lm = reinterpret_cast<double*>(rec + R.lm);
    for (int e = threadIdx.x; e < 3 * L; e += BA_THREADS) lm[e] = out[OL.lm + e];
    double* vel = reinterpret_cast<double*>(rec + R.vel);
    for (int e = threadIdx.x; e < 3 * K; e += BA_THREADS) vel[e] = out[OL.vel + e];
    double* bias = reinterpret_cast<double*>(rec + R.bias);
    if (threadIdx.x < 6) bias[threadIdx.x] = out[OL.bias + threadIdx.x];
    uint8_t* outl = rec + R.outl;
    for (int q = threadIdx.x; q < N; q += BA_THREADS) outl[P.obs_perm[w.o_obs + q]] = P.out_u8[w.o_obs + q];
    uint8_t* bad = rec + R.bad;
    for (int l = threadIdx.x; l < L; l += BA_THREADS) bad[l] = P.out_bad[w.o_lm + l];
    for (int64_t e = R.bad + L + threadIdx.x; e < rec_bytes; e += BA_THREADS) rec[e] = 0;  // padding
}

hipError_t launch_ba_pack(const BaPools& P, int n, uint8_t* dst, int64_t rec_bytes, hipStream_t stream) {
    hipLaunchKernelGGL(ba_pack_kernel, dim3(n), dim3(BA_THREADS), 0, stream, P, dst, rec_bytes);
    return hipGetLastError();
}

// vio_lie_eval (tests): the window factors' Lie maths, one lane per input, compiled like the factors
__global__ void lie_ba_kernel(int op, const double* in, double* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (op == VIO_LIE_SO3_EXP) {
        so3_exp(in + 3 * i, out + 9 * i);
    } else if (op == VIO_LIE_SE3_EXP) {
        se3_exp(in + 6 * i, out + 12 * i, out + 12 * i + 9);
    } else {
        imu_log(in + 9 * i, out + 3 * i);
    }
}
hipError_t launch_lie_ba(int op, const double* in, double* out, int n, hipStream_t stream) {
    hipLaunchKernelGGL(lie_ba_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, op, in, out, n);
    return hipGetLastError();
}

size_t ba_shared_bytes() { return sizeof(BaShared); }
size_t ba_ws_extra_doubles() { return ba_ws_extra(); }
#endif

// kernel attributes are per device: one flag per device ordinal (the caller has selected the
// context's device).  Contexts on one device may live on different host threads (one vio_ctx per
// thread): the flags are read and set under one lock, so no thread launches before the attribute
// call that another thread started has returned.
constexpr int kMaxDevices = 64;
static int current_device() {
    int d = 0;
    return hipGetDevice(&d) == hipSuccess && d >= 0 && d < kMaxDevices ? d : 0;
}
static std::mutex g_attr_mutex;

#ifndef VIO_BA_CLUSTER_TU
hipError_t launch_ba_windows(const BaPools& P, int n, hipStream_t stream) {
    {
        static bool attr_set[kMaxDevices] = {};
        std::lock_guard<std::mutex> lock(g_attr_mutex);
        const int dev = current_device();
        if (!attr_set[dev]) {
            hipError_t e = hipFuncSetAttribute((const void*)ba_window_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)sizeof(BaShared));
            if (e != hipSuccess) return e;
            attr_set[dev] = true;
        }
    }
    hipLaunchKernelGGL(ba_window_kernel, dim3(n), dim3(BA_THREADS), sizeof(BaShared), stream, P);
    return hipGetLastError();
}

#endif
}  // namespace vio360

#include "ba_phases.inc"
#ifndef VIO_BA_CLUSTER_TU
#include "gba_imu.inc"
#endif
