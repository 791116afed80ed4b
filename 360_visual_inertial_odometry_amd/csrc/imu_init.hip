// imu_init.hip — IMU initialisation on device: Optimizer::OptimizeIMUInit
// (src/optimization/Optimizer.cpp:972-1257), one workgroup (one wave) per problem.
//
//   stage 1: gravity direction (theta_x, theta_y) + scale over InertialGravityScaleFactor
//            (src/optimization/Factors.cpp:981-1293), HuberLoss(sqrt(16)), poses / velocities /
//            biases constant;
//   stage 2: velocities + shared biases, the same factors plus two BiasPriorFactor
//            (Factors.h:366-396), gravity direction / scale constant;
//   both: Ceres 2.0 LM (TrustRegionMinimizer + LevenbergMarquardtStrategy, Jacobi scaling,
//         default tolerances) with DENSE_QR (Householder QR of [J~; D]).
// The pose blocks are constant zero perturbations that the factor maps through SE3d::exp without
// the keyframe poses, so every factor sees identity poses (Factors.cpp:1024-1042 with
// Optimizer.cpp:1084-1092); the factor's square-root information is never applied.
//
// The arithmetic follows oracle/ba_oracle.c (oracle_imu_init) operation for operation: sums over
// rows / factors run sequentially in one lane in the oracle's order, the lanes split independent
// columns / factors.  Compiled with -ffp-contract=off like the oracle.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "ctx.h"
#include "lie_dev.h"
#include "vio360.h"

namespace vio360 {
namespace {

constexpr int kThreads = 64;
constexpr int kMaxFrames = 64;
constexpr int kMaxN = 3 * kMaxFrames + 6;

struct IiFactor {  // one InertialGravityScaleFactor (f32 preintegration cast to f64)
    double dR[9], dV[3], dP[3], JRg[9], JVg[9], JVa[9], JPg[9], JPa[9], bg0[3], ba0[3], dt;
    int32_t i, _p;
};

struct IiProb {
    int32_t F, nf, max_it, n2;        // frames, factors, LM iterations per stage, stage-2 parameters
    int32_t m2, _p0;
    int64_t fac;                      // first factor in the factor array
    int64_t vinit;                    // 3F doubles: initial velocities (R_wb_prev * delta_V)
    int64_t scratch;                  // first double of the problem's scratch
    double gm, huber, prior_w;
};

struct IiOut {
    int32_t success, status, it[2], term[2];
    double gravity[3], Rwg[9], gdir[2], scale, bg[3], ba[3], init_cost, final_cost;
};

// ------------------------------------------------------------------------------------------
// maths (oracle: so3d_log, igs_log_so3, igs_right_jac, inv3_eigen, igs_gdir_rot)
__device__ void ii_so3d_log(const double* R, double* w) {
    const double tr = R[0] + R[4] + R[8];
    const double c = fmax(-1.0, fmin(1.0, (tr - 1.0) * 0.5));
    const double th = acos(c);
    if (th < 1e-10) {
        w[0] = R[7]; w[1] = R[2]; w[2] = R[3];
        return;
    }
    const double s = sin(th);
    if (fabs(s) < 1e-10) {
        int mi = 0;
        if (R[4] > R[0]) mi = 1;
        if (R[8] > R[4 * mi]) mi = 2;
        double ax[3];
        ax[mi] = sqrt((R[4 * mi] + 1.0) * 0.5);
        for (int i = 0; i < 3; ++i)
            if (i != mi) ax[i] = R[3 * mi + i] / (2.0 * ax[mi]);
        const double sk[3] = {(R[7] - R[5]) * 0.5, (R[2] - R[6]) * 0.5, (R[3] - R[1]) * 0.5};
        if (ax[0] * sk[0] + ax[1] * sk[1] + ax[2] * sk[2] < 0) { ax[0] = -ax[0]; ax[1] = -ax[1]; ax[2] = -ax[2]; }
        w[0] = ax[0] * th; w[1] = ax[1] * th; w[2] = ax[2] * th;
        return;
    }
    const double f = th / (2.0 * s);
    w[0] = f * (R[7] - R[5]); w[1] = f * (R[2] - R[6]); w[2] = f * (R[3] - R[1]);
}

__device__ void ii_log_so3(const double* R, double* w) {
    double R1[9], R2[9];
    polar3(R, R1);
    polar3(R1, R2);
    ii_so3d_log(R2, w);
}

__device__ void ii_right_jac(const double* phi, double* J) {
    double P[9];
    hat3(phi, P);
    const double th = nrm3(phi);
    if (th < 1e-6) {
        for (int i = 0; i < 9; ++i) J[i] = ((i % 4 == 0) ? 1.0 : 0.0) - 0.5 * P[i];
        return;
    }
    double P2[9];
    m3mul(P, P, P2);
    const double c = cos(th), s = sin(th);
    for (int i = 0; i < 9; ++i)
        J[i] = ((i % 4 == 0) ? 1.0 : 0.0) - P[i] * (1.0 - c) / (th * th) + P2[i] * (th - s) / (th * th * th);
}

__device__ void ii_inv3(const double* m, double* r) {
    auto M = [&](int i, int j) { return m[3 * i + j]; };
    auto cof = [&](int i, int j) {
        return M((i + 1) % 3, (j + 1) % 3) * M((i + 2) % 3, (j + 2) % 3) -
               M((i + 1) % 3, (j + 2) % 3) * M((i + 2) % 3, (j + 1) % 3);
    };
    const double c0[3] = {cof(0, 0), cof(1, 0), cof(2, 0)};
    const double det = c0[0] * M(0, 0) + c0[1] * M(1, 0) + c0[2] * M(2, 0);
    const double id = 1.0 / det;
    for (int j = 0; j < 3; ++j) r[j] = c0[j] * id;
    for (int i = 1; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[3 * i + j] = cof(j, i) * id;
}

__device__ void ii_gdir_rot(const double* gd, double* R) {
    const double w[3] = {gd[0], gd[1], 0.0};
    const double d2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    const double d = sqrt(d2);
    double W[9], W2[9];
    hat3(w, W);
    m3mul(W, W, W2);
    for (int i = 0; i < 9; ++i) {
        const double I = (i % 4 == 0) ? 1.0 : 0.0;
        R[i] = d < 1e-5 ? I + W[i] + 0.5 * W2[i] : I + W[i] * sin(d) / d + W2[i] * (1.0 - cos(d)) / d2;
    }
}

// SO3d::Exp followed by the SO3d constructor's projection (oracle so3_exp)
__device__ void ii_so3_exp(const double* w, double* R) {
    double M[9];
    so3_exp(w, M);
    polar3(M, R);
}

// ------------------------------------------------------------------------------------------
struct IiParams {  // parameter values of the current evaluation
    const double* vel;  // 3F
    double bg[3], ba[3], gdir[2], scale;
};

// InertialGravityScaleFactor::Evaluate at identity poses (oracle igs_eval_factor).  B: 9x3 blocks
// vel_i, bg, ba, vel_j (27 each), then gravity_dir 9x2 (18), scale 9x1 (9).
__device__ void ii_factor(const IiParams& P, const IiFactor& f, double gm, double* r, double* B) {
    const double* vi = P.vel + 3 * f.i;
    const double* vj = P.vel + 3 * (f.i + 1);
    const double s = P.scale, dt = f.dt;
    double Rwg[9], g[3];
    ii_gdir_rot(P.gdir, Rwg);
    for (int k = 0; k < 3; ++k) g[k] = Rwg[3 * k + 2] * -gm;
    double dR[9], dV[3], dP[3], dbg[3], dba[3];
    for (int k = 0; k < 9; ++k) dR[k] = f.dR[k];
    for (int k = 0; k < 3; ++k) {
        dV[k] = f.dV[k]; dP[k] = f.dP[k];
        dbg[k] = P.bg[k] - f.bg0[k];
        dba[k] = P.ba[k] - f.ba0[k];
    }
    if (nrm3(dbg) > 1e-6 || nrm3(dba) > 1e-6) {
        double w[3], E[9], M[9], a[3], b[3];
        m3vec(f.JRg, dbg, w);
        ii_so3_exp(w, E);
        m3mul(dR, E, M);
        for (int k = 0; k < 9; ++k) dR[k] = M[k];
        m3vec(f.JVg, dbg, a); m3vec(f.JVa, dba, b);
        for (int k = 0; k < 3; ++k) dV[k] = dV[k] + a[k] + b[k];
        m3vec(f.JPg, dbg, a); m3vec(f.JPa, dba, b);
        for (int k = 0; k < 3; ++k) dP[k] = dP[k] + a[k] + b[k];
    }
    double eR[9], er[3];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) eR[3 * a + b] = dR[3 * b + a];
    ii_log_so3(eR, er);
    for (int k = 0; k < 3; ++k) {
        r[k] = er[k];
        r[3 + k] = (s * (vj[k] - vi[k]) - g[k] * dt) - dV[k];
        r[6 + k] = (s * (0.0 - vi[k] * dt) - 0.5 * g[k] * dt * dt) - dP[k];
    }
    if (!B) return;
    for (int k = 0; k < 4 * 27 + 18 + 9; ++k) B[k] = 0.0;
    double* Jvi = B;
    double* Jbg = B + 27;
    double* Jba = B + 54;
    double* Jvj = B + 81;
    double* Jgd = B + 108;
    double* Jsc = B + 126;
    for (int k = 0; k < 3; ++k) {
        Jvi[3 * (3 + k) + k] = -s;
        Jvi[3 * (6 + k) + k] = -s * dt;
        Jvj[3 * (3 + k) + k] = s;
    }
    double Jr[9], Jri[9], Jb[9], t1[9], t2[9], t3[9], w[3], eRt[9];
    ii_right_jac(er, Jr);
    ii_inv3(Jr, Jri);
    m3vec(f.JRg, dbg, w);
    ii_right_jac(w, Jb);
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) eRt[3 * a + b] = eR[3 * b + a];
    for (int i = 0; i < 9; ++i) t1[i] = -Jri[i];
    m3mul(t1, eRt, t2);
    m3mul(t2, Jb, t3);
    m3mul(t3, f.JRg, t1);
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
            Jbg[3 * a + b] = t1[3 * a + b];
            Jbg[3 * (3 + a) + b] = -f.JVg[3 * a + b];
            Jbg[3 * (6 + a) + b] = -f.JPg[3 * a + b];
            Jba[3 * (3 + a) + b] = -f.JVa[3 * a + b];
            Jba[3 * (6 + a) + b] = -f.JPa[3 * a + b];
        }
    for (int k = 0; k < 3; ++k) {
        const double d0 = Rwg[3 * k + 1] * gm, d1 = Rwg[3 * k] * -gm;
        Jgd[2 * (3 + k)] = -d0 * dt;
        Jgd[2 * (3 + k) + 1] = -d1 * dt;
        Jgd[2 * (6 + k)] = -0.5 * d0 * dt * dt;
        Jgd[2 * (6 + k) + 1] = -0.5 * d1 * dt * dt;
        Jsc[3 + k] = vj[k] - vi[k];
        Jsc[6 + k] = 0.0 - vi[k] * dt;
    }
}

// Huber(delta) rho and the Corrector's sqrt(rho') (rho'' <= 0: alpha = 0, corrector.cc:82-86)
__device__ __forceinline__ void ii_huber(double delta, double s, double& rho0, double& sr1) {
    const double b = delta * delta, a = delta;
    if (s > b) {
        const double r = sqrt(s);
        rho0 = 2.0 * a * r - b;
        sr1 = sqrt(fmax(DBL_MIN, a / r));
    } else {
        rho0 = s;
        sr1 = sqrt(1.0);
    }
}

struct IiShared {
    double x[kMaxN], xu[kMaxN], cand[kMaxN], g[kMaxN], colsq[kMaxN], s[kMaxN], D[kMaxN], y[kMaxN];
    double vel[3 * kMaxFrames];
    double bg[3], ba[3], gdir[2], scale;
    double fcost[kMaxFrames];
    double bc[4];  // lane-0 results broadcast to the wave
    int vel_off[kMaxFrames];
    int bg_off, ba_off;
};

struct IiWork {  // the problem's global scratch
    double* J;   // m x n row-major
    double* r;   // m
    double* A;   // (m + n) x n column-major
    double* b;   // m + n
    double* v;   // m + n
    double* jh;  // m
};

// x -> the parameter state (oracle igs_unpack)
__device__ void ii_unpack(IiShared& S, int stage, int F, const double* xv) {
    const int t = threadIdx.x;
    __syncthreads();
    if (stage == 1) {
        if (t == 0) { S.gdir[0] = xv[0]; S.gdir[1] = xv[1]; S.scale = xv[2]; }
    } else {
        for (int k = t; k < F; k += kThreads)
            if (S.vel_off[k] >= 0)
                for (int c = 0; c < 3; ++c) S.vel[3 * k + c] = xv[S.vel_off[k] + c];
        if (t < 3) { S.bg[t] = xv[S.bg_off + t]; S.ba[t] = xv[S.ba_off + t]; }
    }
    __syncthreads();
}

// oracle igs_eval: the cost (every lane); with want_jac the corrected J / r and g = J^T r, colsq
__device__ double ii_eval(IiShared& S, const IiProb& p, const IiFactor* fac, int stage, int n, int m,
                          const double* xv, bool want_jac, const IiWork& w) {
    const int t = threadIdx.x;
    ii_unpack(S, stage, p.F, xv);
    IiParams P;
    P.vel = S.vel;
    for (int k = 0; k < 3; ++k) { P.bg[k] = S.bg[k]; P.ba[k] = S.ba[k]; }
    P.gdir[0] = S.gdir[0]; P.gdir[1] = S.gdir[1]; P.scale = S.scale;
    for (int q = t; q < p.nf; q += kThreads) {
        const IiFactor& f = fac[q];
        double r[9], B[4 * 27 + 18 + 9];
        ii_factor(P, f, p.gm, r, want_jac ? B : nullptr);
        double sq = 0;
        for (int i = 0; i < 9; ++i) sq += r[i] * r[i];
        double rho0, sr1;
        ii_huber(p.huber, sq, rho0, sr1);
        S.fcost[q] = 0.5 * rho0;
        if (want_jac) {
            double* row = w.J + (size_t)9 * q * n;
            for (int e = 0; e < 9 * n; ++e) row[e] = 0.0;
            if (stage == 1) {
                for (int i = 0; i < 9; ++i) {
                    row[i * n] = B[108 + 2 * i] * sr1;
                    row[i * n + 1] = B[108 + 2 * i + 1] * sr1;
                    row[i * n + 2] = B[126 + i] * sr1;
                }
            } else {
                const int offs[4] = {S.vel_off[f.i], S.bg_off, S.ba_off, S.vel_off[f.i + 1]};
                for (int b = 0; b < 4; ++b)
                    for (int i = 0; i < 9; ++i)
                        for (int j = 0; j < 3; ++j) row[i * n + offs[b] + j] = B[27 * b + 3 * i + j] * sr1;
            }
            for (int i = 0; i < 9; ++i) w.r[9 * q + i] = r[i] * sr1;
        }
    }
    __syncthreads();
    if (t == 0) {
        double total = 0.0;
        for (int q = 0; q < p.nf; ++q) total += S.fcost[q];
        if (stage == 2) {
            for (int b = 0; b < 2; ++b) {  // BiasPriorFactor (gyro, then accel), no loss
                const double* v = b ? S.ba : S.bg;
                const int off = b ? S.ba_off : S.bg_off;
                double sq = 0, rr[3];
                for (int k = 0; k < 3; ++k) { rr[k] = p.prior_w * (v[k] - 0.0); sq += rr[k] * rr[k]; }
                total += 0.5 * sq;
                if (want_jac) {
                    const int row0 = 9 * p.nf + 3 * b;
                    for (int k = 0; k < 3; ++k) {
                        for (int j = 0; j < n; ++j) w.J[(size_t)(row0 + k) * n + j] = 0.0;
                        w.J[(size_t)(row0 + k) * n + off + k] = p.prior_w;
                        w.r[row0 + k] = rr[k];
                    }
                }
            }
        }
        S.bc[0] = total;
    }
    __syncthreads();
    if (want_jac) {
        for (int j = t; j < n; j += kThreads) {
            double gj = 0.0, cj = 0.0;
            for (int i = 0; i < m; ++i) {
                const double a = w.J[(size_t)i * n + j];
                gj += a * w.r[i];
                cj += a * a;
            }
            S.g[j] = gj;
            S.colsq[j] = cj;
        }
    }
    const double total = S.bc[0];
    __syncthreads();
    return total;
}

// DENSE_QR: y = argmin |J~ y - r|^2 + |D y|^2 with J~ = J diag(s) (oracle igs_solve +
// dense_qr_lm_solve); returns false on a zero column
__device__ bool ii_solve(IiShared& S, int n, int m, const IiWork& w) {
    const int t = threadIdx.x;
    const int R = m + n;
    for (int c = t; c < n; c += kThreads) {
        double* col = w.A + (size_t)c * R;
        for (int i = 0; i < m; ++i) col[i] = w.J[(size_t)i * n + c] * S.s[c];
        for (int i = 0; i < n; ++i) col[m + i] = (i == c) ? S.D[c] : 0.0;
    }
    for (int i = t; i < R; i += kThreads) w.b[i] = i < m ? w.r[i] : 0.0;
    __syncthreads();
    for (int j = 0; j < n; ++j) {
        const double* cj = w.A + (size_t)j * R;
        if (t == 0) {
            double nrm = 0;
            for (int i = j; i < R; ++i) nrm += cj[i] * cj[i];
            nrm = sqrt(nrm);
            double vn = 0;
            if (nrm != 0.0) {
                const double alpha = cj[j] > 0 ? -nrm : nrm;
                for (int i = j; i < R; ++i) w.v[i] = cj[i];
                w.v[j] -= alpha;
                for (int i = j; i < R; ++i) vn += w.v[i] * w.v[i];
            }
            S.bc[1] = nrm;
            S.bc[2] = vn;
        }
        __syncthreads();
        if (S.bc[1] == 0.0) return false;  // uniform: every lane leaves
        const double vn = S.bc[2];
        if (vn != 0.0) {
            for (int c = j + t; c <= n; c += kThreads) {  // c == n: the right-hand side
                double* col = c < n ? w.A + (size_t)c * R : w.b;
                double d = 0;
                for (int i = j; i < R; ++i) d += w.v[i] * col[i];
                d = 2.0 * d / vn;
                for (int i = j; i < R; ++i) col[i] -= d * w.v[i];
            }
        }
        __syncthreads();
    }
    if (t == 0)
        for (int j = n - 1; j >= 0; --j) {
            double tt = w.b[j];
            for (int c = j + 1; c < n; ++c) tt -= w.A[(size_t)c * R + j] * S.y[c];
            S.y[j] = tt / w.A[(size_t)j * R + j];
        }
    __syncthreads();
    return true;
}

// model cost change -(J~ h)^T (r + J~ h / 2) (oracle igs_model); every lane returns it
__device__ double ii_model(IiShared& S, int n, int m, const IiWork& w) {
    const int t = threadIdx.x;
    for (int i = t; i < m; i += kThreads) {
        double jh = 0;
        for (int j = 0; j < n; ++j) jh += w.J[(size_t)i * n + j] * (S.s[j] * S.y[j]);
        w.jh[i] = jh;
    }
    __syncthreads();
    if (t == 0) {
        double mc = 0;
        for (int i = 0; i < m; ++i) mc -= w.jh[i] * (w.r[i] + w.jh[i] / 2.0);
        S.bc[3] = mc;
    }
    __syncthreads();
    const double mc = S.bc[3];
    __syncthreads();
    return mc;
}

struct IiStage {
    int iterations, termination;
    double initial_cost, final_cost;
};

// oracle_lm_minimize (TrustRegionMinimizer + LevenbergMarquardtStrategy, default options) on the
// stage's parameter vector S.x; the solution Ceres copies back ends in S.x
__device__ IiStage ii_minimize(IiShared& S, const IiProb& p, const IiFactor* fac, int stage, int n, int m,
                               const IiWork& w) {
    const int t = threadIdx.x;
    const double ftol = 1e-6, gtol = 1e-10, ptol = 1e-8, max_radius = 1e16, min_radius = 1e-32;
    const double min_rel = 1e-3, dmin = 1e-6, dmax = 1e32;
    IiStage out{0, VIO_TERM_NO_CONVERGENCE, 0.0, 0.0};
    for (int i = t; i < n; i += kThreads) S.xu[i] = S.x[i];  // x_user (the best point so far)
    __syncthreads();
    double x_norm = -1.0, x_cost = DBL_MAX, minimum_cost = DBL_MAX;
    double radius = 1e4, decrease = 2.0;
    int consecutive_invalid = 0;
    x_cost = ii_eval(S, p, fac, stage, n, m, S.x, true, w);
    for (int i = t; i < n; i += kThreads) S.s[i] = 1.0 / (1.0 + sqrt(S.colsq[i]));
    __syncthreads();
    auto grad_max = [&]() {
        if (t == 0) {
            double gm = 0.0;
            for (int i = 0; i < n; ++i) gm = fmax(gm, fabs(S.x[i] - (S.x[i] + (-S.g[i]))));
            S.bc[1] = gm;
        }
        __syncthreads();
        const double v = S.bc[1];
        __syncthreads();
        return v;
    };
    double gmax = grad_max();
    out.initial_cost = x_cost;
    double step_eval_current = x_cost;
    int iteration = 0;
    bool step_successful = true;
    double iter_cost = x_cost, final_cost = x_cost;
    for (;;) {
        if (step_successful) {
            if (x_cost < minimum_cost) {
                minimum_cost = x_cost;
                for (int i = t; i < n; i += kThreads) S.xu[i] = S.x[i];
            }
        }
        out.iterations++;
        final_cost = fmin(final_cost, iter_cost);
        if (iteration >= p.max_it) { out.termination = VIO_TERM_NO_CONVERGENCE; break; }
        if (step_successful && gmax <= gtol) { out.termination = VIO_TERM_CONVERGENCE; break; }
        if (radius <= min_radius) { out.termination = VIO_TERM_CONVERGENCE; break; }
        iteration++;
        for (int i = t; i < n; i += kThreads) {
            double d = S.colsq[i] * S.s[i] * S.s[i];
            d = fmin(fmax(d, dmin), dmax);
            S.D[i] = sqrt(d / radius);
        }
        __syncthreads();
        bool valid = ii_solve(S, n, m, w);
        if (valid && t == 0) {
            int fin = 1;
            for (int i = 0; i < n; ++i)
                if (!isfinite(S.y[i])) fin = 0;
            S.bc[1] = fin;
        }
        __syncthreads();
        if (valid) valid = S.bc[1] != 0.0;
        __syncthreads();
        double model_change = 0.0;
        if (valid) {
            for (int i = t; i < n; i += kThreads) S.y[i] = -S.y[i];
            __syncthreads();
            model_change = ii_model(S, n, m, w);
            valid = model_change > 0.0;
        }
        if (!valid) {
            if (++consecutive_invalid >= 5) { out.termination = VIO_TERM_FAILURE; break; }
            radius = radius / decrease;
            decrease *= 2.0;
            step_successful = false;
            iter_cost = x_cost;
            continue;
        }
        consecutive_invalid = 0;
        for (int i = t; i < n; i += kThreads) S.cand[i] = S.x[i] + S.y[i] * S.s[i];
        __syncthreads();
        const double cand_cost = ii_eval(S, p, fac, stage, n, m, S.cand, false, w);
        if (t == 0) {
            double sn = 0;
            for (int i = 0; i < n; ++i) { const double d = S.x[i] - S.cand[i]; sn += d * d; }
            S.bc[1] = sqrt(sn);
        }
        __syncthreads();
        const double step_norm = S.bc[1];
        __syncthreads();
        if (step_norm <= ptol * (x_norm + ptol)) { out.termination = VIO_TERM_CONVERGENCE; break; }
        if (fabs(x_cost - cand_cost) <= ftol * x_cost) { out.termination = VIO_TERM_CONVERGENCE; break; }
        const double rel = cand_cost >= DBL_MAX ? -DBL_MAX : (step_eval_current - cand_cost) / model_change;
        if (rel > min_rel) {
            for (int i = t; i < n; i += kThreads) S.x[i] = S.cand[i];
            __syncthreads();
            if (t == 0) {
                double xn = 0;
                for (int i = 0; i < n; ++i) xn += S.x[i] * S.x[i];
                S.bc[1] = sqrt(xn);
            }
            __syncthreads();
            x_norm = S.bc[1];
            __syncthreads();
            x_cost = ii_eval(S, p, fac, stage, n, m, S.x, true, w);
            gmax = grad_max();
            step_successful = true;
            radius = radius / fmax(1.0 / 3.0, 1.0 - pow(2.0 * rel - 1.0, 3));
            radius = fmin(max_radius, radius);
            decrease = 2.0;
            step_eval_current = cand_cost;
            iter_cost = x_cost;
        } else {
            step_successful = false;
            iter_cost = cand_cost;
            radius = radius / decrease;
            decrease *= 2.0;
        }
    }
    out.final_cost = final_cost;
    __syncthreads();
    // the point Ceres copies back (the initial one after a failure, oracle `done:`)
    if (out.termination != VIO_TERM_FAILURE)
        for (int i = t; i < n; i += kThreads) S.x[i] = S.xu[i];
    __syncthreads();
    return out;
}

__global__ __launch_bounds__(kThreads) void imu_init_kernel(const IiProb* __restrict__ probs,
                                                            const IiFactor* __restrict__ facs,
                                                            const double* __restrict__ vinit,
                                                            double* __restrict__ scratch, IiOut* __restrict__ outs,
                                                            double* __restrict__ vel_out) {
    __shared__ IiShared S;
    const IiProb p = probs[blockIdx.x];
    const IiFactor* fac = facs + p.fac;
    const int t = threadIdx.x;
    const int F = p.F;
    double* base = scratch + p.scratch;
    IiWork w;
    w.J = base;
    w.r = w.J + (size_t)p.m2 * p.n2;
    w.A = w.r + p.m2;
    w.b = w.A + (size_t)(p.m2 + p.n2) * p.n2;
    w.v = w.b + p.m2 + p.n2;
    w.jh = w.v + p.m2 + p.n2;
    for (int k = t; k < 3 * F; k += kThreads) S.vel[k] = vinit[p.vinit + k];
    if (t == 0) {
        for (int k = 0; k < 3; ++k) { S.bg[k] = 0.0; S.ba[k] = 0.0; }
        S.gdir[0] = S.gdir[1] = 0.0;
        S.scale = 1.0;
        // stage-2 layout: velocities and biases in order of first appearance (Ceres program order)
        for (int k = 0; k < F; ++k) S.vel_off[k] = -1;
        S.bg_off = S.ba_off = -1;
        int off = 0;
        for (int q = 0; q < p.nf; ++q) {
            const int i = fac[q].i;
            if (S.vel_off[i] < 0) { S.vel_off[i] = off; off += 3; }
            if (S.bg_off < 0) { S.bg_off = off; off += 3; }
            if (S.ba_off < 0) { S.ba_off = off; off += 3; }
            if (S.vel_off[i + 1] < 0) { S.vel_off[i + 1] = off; off += 3; }
        }
        S.x[0] = S.x[1] = 0.0;
        S.x[2] = 1.0;
    }
    __syncthreads();
    // stage 1: gravity direction + scale
    const IiStage s1 = ii_minimize(S, p, fac, 1, 3, 9 * p.nf, w);
    ii_unpack(S, 1, F, S.x);
    // stage 2: velocities + biases
    for (int k = t; k < F; k += kThreads)
        if (S.vel_off[k] >= 0)
            for (int c = 0; c < 3; ++c) S.x[S.vel_off[k] + c] = S.vel[3 * k + c];
    if (t < 3) { S.x[S.bg_off + t] = S.bg[t]; S.x[S.ba_off + t] = S.ba[t]; }
    __syncthreads();
    const IiStage s2 = ii_minimize(S, p, fac, 2, p.n2, p.m2, w);
    ii_unpack(S, 2, F, S.x);
    if (t == 0) {
        IiOut o;
        o.success = 1;
        o.status = VIO_IMU_INIT_OK;
        o.it[0] = s1.iterations; o.it[1] = s2.iterations;
        o.term[0] = s1.termination; o.term[1] = s2.termination;
        o.init_cost = s1.initial_cost;
        o.final_cost = s2.final_cost;
        // AngleAxisd(|w|, w / |w|).toRotationMatrix() for w = (theta_x, theta_y, 0) (:1212-1224)
        const double om[3] = {S.gdir[0], S.gdir[1], 0.0};
        const double ang = sqrt(om[0] * om[0] + om[1] * om[1] + om[2] * om[2]);
        double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        if (!(ang < 1e-6)) {
            const double ax[3] = {om[0] / ang, om[1] / ang, om[2] / ang};
            const double sn = sin(ang), cs = cos(ang);
            const double sa[3] = {sn * ax[0], sn * ax[1], sn * ax[2]};
            const double ca[3] = {(1.0 - cs) * ax[0], (1.0 - cs) * ax[1], (1.0 - cs) * ax[2]};
            double tt = ca[0] * ax[1];
            R[1] = tt - sa[2]; R[3] = tt + sa[2];
            tt = ca[0] * ax[2];
            R[2] = tt + sa[1]; R[6] = tt - sa[1];
            tt = ca[1] * ax[2];
            R[5] = tt - sa[0]; R[7] = tt + sa[0];
            R[0] = ca[0] * ax[0] + cs; R[4] = ca[1] * ax[1] + cs; R[8] = ca[2] * ax[2] + cs;
        }
        for (int k = 0; k < 9; ++k) o.Rwg[k] = R[k];
        for (int k = 0; k < 3; ++k) o.gravity[k] = R[3 * k + 2] * -9.81;
        o.gdir[0] = S.gdir[0]; o.gdir[1] = S.gdir[1];
        o.scale = S.scale;
        for (int k = 0; k < 3; ++k) { o.bg[k] = S.bg[k]; o.ba[k] = S.ba[k]; }
        outs[blockIdx.x] = o;
    }
    for (int k = t; k < 3 * F; k += kThreads) vel_out[p.vinit + k] = S.vel[k];
}

// vio_lie_eval (tests): SO3d::Exp with its projection and SO3d::Log, one lane per input
__global__ void lie_init_kernel(int op, const double* in, double* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (op == VIO_LIE_SO3D_EXP) ii_so3_exp(in + 3 * i, out + 9 * i);
    else ii_so3d_log(in + 9 * i, out + 3 * i);
}

}  // namespace

hipError_t launch_lie_init(int op, const double* in, double* out, int n, hipStream_t stream) {
    hipLaunchKernelGGL(lie_init_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, op, in, out, n);
    return hipGetLastError();
}
}  // namespace vio360

using namespace vio360;

// status of one problem on the host (the guards of :977-989 and the stage-1 factor count)
static int imu_init_status(const vio_imu_init_problem& p, int* nf) {
    *nf = 0;
    if (p.num_frames < 3) return VIO_IMU_INIT_FEW_FRAMES;
    for (int i = 1; i < p.num_frames; ++i)
        if (!p.preint_valid[i]) return VIO_IMU_INIT_NO_PREINT;
    for (int i = 0; i < p.num_frames - 1; ++i) {
        const double dt = p.preint[i + 1].dt_total;
        if (!(dt < 0.001 || dt > 2.0)) ++*nf;
    }
    return *nf ? VIO_IMU_INIT_OK : VIO_IMU_INIT_NO_FACTORS;
}

static void imu_init_default(vio_imu_init_result* r, int status) {
    double* v = r->velocities;
    std::memset(r, 0, sizeof *r);
    r->velocities = v;
    r->status = status;
    r->scale = 1.0;
    r->gravity[2] = (double)-9.81f;  // IMUInitResult() defaults
    r->Rwg[0] = r->Rwg[4] = r->Rwg[8] = 1.0;
}

extern "C" int vio_imu_init_solve(vio_ctx* ctx, const vio_imu_init_problem* probs, vio_imu_init_result* res, int n) {
    if (!ctx || n < 0 || (n > 0 && (!probs || !res))) return VIO_EINVAL;
    std::vector<IiProb> hp;
    std::vector<IiFactor> hf;
    std::vector<double> hv;
    std::vector<int> slot(n, -1);
    size_t scratch = 0;
    for (int k = 0; k < n; ++k) {
        const vio_imu_init_problem& p = probs[k];
        if (p.num_frames > kMaxFrames || p.num_frames < 0 || (p.num_frames > 0 && (!p.preint || !p.preint_valid || !p.T_wb))) {
            set_error(ctx, "vio_imu_init_solve: num_frames must be <= 64 with preint / preint_valid / T_wb given");
            return VIO_EINVAL;
        }
        int nf = 0;
        const int st = imu_init_status(p, &nf);
        imu_init_default(&res[k], st);
        if (st != VIO_IMU_INIT_OK) continue;
        IiProb q{};
        q.F = p.num_frames;
        q.nf = nf;
        q.max_it = p.max_iterations;
        q.fac = (int64_t)hf.size();
        q.vinit = (int64_t)hv.size();
        q.gm = p.gravity_magnitude;
        q.huber = p.huber_delta;
        q.prior_w = p.bias_prior_weight;
        // velocity initialisation R_wb_prev * delta_V (:1025-1036), the oracle's m3_vec order
        for (int i = 0; i < p.num_frames; ++i) {
            double v[3] = {0.0, 0.0, 0.0};
            if (i > 0 && p.preint[i].dt_total > 0.001) {
                const double* R = p.T_wb[i - 1].R;
                const double dv[3] = {p.preint[i].delta_V[0], p.preint[i].delta_V[1], p.preint[i].delta_V[2]};
                for (int a = 0; a < 3; ++a) v[a] = R[3 * a] * dv[0] + R[3 * a + 1] * dv[1] + R[3 * a + 2] * dv[2];
            }
            hv.insert(hv.end(), v, v + 3);
        }
        uint8_t seen[kMaxFrames] = {0};
        int n2 = 6;
        for (int i = 0; i < p.num_frames - 1; ++i) {
            const vio_preint& pr = p.preint[i + 1];
            if (pr.dt_total < 0.001 || pr.dt_total > 2.0) continue;
            IiFactor f{};
            f.i = i;
            f.dt = pr.dt_total;
            for (int e = 0; e < 9; ++e) {
                f.dR[e] = pr.delta_R[e];
                f.JRg[e] = pr.J_Rg[e]; f.JVg[e] = pr.J_Vg[e]; f.JVa[e] = pr.J_Va[e];
                f.JPg[e] = pr.J_Pg[e]; f.JPa[e] = pr.J_Pa[e];
            }
            for (int e = 0; e < 3; ++e) {
                f.dV[e] = pr.delta_V[e]; f.dP[e] = pr.delta_P[e];
                f.bg0[e] = pr.gyro_bias[e]; f.ba0[e] = pr.accel_bias[e];
            }
            hf.push_back(f);
            for (int e : {i, i + 1})
                if (!seen[e]) { seen[e] = 1; n2 += 3; }
        }
        q.n2 = n2;
        q.m2 = 9 * nf + 6;
        q.scratch = (int64_t)scratch;
        const size_t m2 = q.m2, nn = q.n2;
        scratch += m2 * nn + m2 + (m2 + nn) * nn + 2 * (m2 + nn) + m2;
        scratch = (scratch + 31) & ~size_t(31);
        slot[k] = (int)hp.size();
        hp.push_back(q);
    }
    if (hp.empty()) return VIO_OK;
    const size_t b_p = ((sizeof(IiProb) * hp.size()) + 255) & ~size_t(255);
    const size_t b_f = ((sizeof(IiFactor) * hf.size()) + 255) & ~size_t(255);
    const size_t b_v = ((sizeof(double) * hv.size()) + 255) & ~size_t(255);
    const size_t b_o = ((sizeof(IiOut) * hp.size()) + 255) & ~size_t(255);
    const size_t b_s = sizeof(double) * scratch;
    VIO_DEVICE(ctx);
    auto* d = static_cast<char*>(ctx_buffer(ctx, kSlotImuInit, b_p + b_f + 2 * b_v + b_o + b_s));
    if (!d) {
        set_error(ctx, "vio_imu_init_solve: device allocation failed");
        return VIO_ENOMEM;
    }
    auto* d_p = reinterpret_cast<IiProb*>(d);
    auto* d_f = reinterpret_cast<IiFactor*>(d + b_p);
    auto* d_v = reinterpret_cast<double*>(d + b_p + b_f);
    auto* d_vo = reinterpret_cast<double*>(d + b_p + b_f + b_v);
    auto* d_o = reinterpret_cast<IiOut*>(d + b_p + b_f + 2 * b_v);
    auto* d_s = reinterpret_cast<double*>(d + b_p + b_f + 2 * b_v + b_o);
    hipStream_t st = ctx->stream;
    VIO_HIP(ctx, hipMemcpyAsync(d_p, hp.data(), sizeof(IiProb) * hp.size(), hipMemcpyHostToDevice, st));
    VIO_HIP(ctx, hipMemcpyAsync(d_f, hf.data(), sizeof(IiFactor) * hf.size(), hipMemcpyHostToDevice, st));
    VIO_HIP(ctx, hipMemcpyAsync(d_v, hv.data(), sizeof(double) * hv.size(), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(imu_init_kernel, dim3((unsigned)hp.size()), dim3(kThreads), 0, st, d_p, d_f, d_v, d_s, d_o,
                       d_vo);
    VIO_HIP(ctx, hipGetLastError());
    std::vector<IiOut> ho(hp.size());
    std::vector<double> hvo(hv.size());
    VIO_HIP(ctx, hipMemcpyAsync(ho.data(), d_o, sizeof(IiOut) * hp.size(), hipMemcpyDeviceToHost, st));
    VIO_HIP(ctx, hipMemcpyAsync(hvo.data(), d_vo, sizeof(double) * hv.size(), hipMemcpyDeviceToHost, st));
    VIO_HIP(ctx, hipStreamSynchronize(st));
    for (int k = 0; k < n; ++k) {
        if (slot[k] < 0) continue;
        const IiOut& o = ho[slot[k]];
        vio_imu_init_result& r = res[k];
        r.success = o.success;
        r.status = o.status;
        for (int e = 0; e < 2; ++e) { r.iterations[e] = o.it[e]; r.termination[e] = o.term[e]; r.gravity_dir[e] = o.gdir[e]; }
        for (int e = 0; e < 3; ++e) { r.gravity[e] = o.gravity[e]; r.gyro_bias[e] = o.bg[e]; r.accel_bias[e] = o.ba[e]; }
        for (int e = 0; e < 9; ++e) r.Rwg[e] = o.Rwg[e];
        r.scale = o.scale;
        r.initial_cost = o.init_cost;
        r.final_cost = o.final_cost;
        if (r.velocities)
            std::memcpy(r.velocities, hvo.data() + hp[slot[k]].vinit, sizeof(double) * 3 * probs[k].num_frames);
    }
    return VIO_OK;
}
