/*
 * ba_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + timed CPU baseline, never shipped).
 *
 * CPU restatement, in plain C99, of the reference's sliding-window bundle-adjustment path:
 *   - ERP reprojection factors  BAFactor / PnPFactor (src/optimization/Factors.cpp:33-612)
 *   - InertialFactorFixedGravity (src/optimization/Factors.cpp:1299-1519)
 *   - SE3d/SO3d maths incl. the SVD re-orthonormalisation (src/util/LieUtils.cpp:203-370)
 *   - HuberLoss + Corrector (thirdparty/ceres-solver/internal/ceres/loss_function.cc:48-62,
 *     corrector.cc:42-156, residual_block.cc:161-197)
 *   - Ceres 2.0 TrustRegionMinimizer + LevenbergMarquardtStrategy with Jacobi scaling
 *     (internal/ceres/trust_region_minimizer.cc:67-826, levenberg_marquardt_strategy.cc:66-160,
 *      trust_region_step_evaluator.cc:52-63), fixed-block removal (program.cc:305-400) and
 *     final-cost bookkeeping (solver_utils.h:46-55)
 *   - Schur-complement linear solve with the points as e-blocks
 *     (internal/ceres/schur_complement_solver.cc:118-356, schur_eliminator_impl.h:179-377)
 *   - Optimizer::RunLocalBA / RunBA / RunVIBA / SolvePnP solve + chi^2 post-processing
 *     (src/optimization/Optimizer.cpp:83-966)
 *
 * It consumes the same vio_ba_problem the HIP library consumes (include/vio360.h) so the two
 * can be compared on identical inputs.  Parity status: the Ceres control flow is pinned by the
 * restated Ceres known-answer tests (tests/test_oracle_kat.py); the first-party factor maths has
 * no reference tests and is cross-checked against an independent numpy restatement
 * (oracle/oracle_np.py) and finite differences — "parity unpinned" against the reference binary,
 * which cannot be built here (no Eigen/OpenCV in the image).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#include <time.h>
#endif

#include "../include/vio360.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

#define EPS_D 1e-10 /* kEpsilonD, src/util/LieUtils.h:24 */

/* Threads of one window solve (the CPU-baseline leg only; Ceres runs num_threads = 4,
   src/optimization/Optimizer.cpp:79).  1 (the default, and what every parity test uses) runs the
   single-threaded code paths unchanged; > 1 switches the observation loops, the Schur elimination
   and the back-substitution to OpenMP variants whose reduction order differs from the serial one. */
static int oracle_threads = 1;
void oracle_set_threads(int n) { oracle_threads = n > 1 ? n : 1; }
int oracle_get_threads(void) { return oracle_threads; }

/* ========================================================================================= */
/* 3x3 helpers (row-major)                                                                   */
/* ========================================================================================= */
static void m3_mul(const double* a, const double* b, double* c) {
    double t[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) t[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
    memcpy(c, t, sizeof t);
}
static void m3_tr(const double* a, double* b) {
    double t[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) t[3 * i + j] = a[3 * j + i];
    memcpy(b, t, sizeof t);
}
static void m3_vec(const double* a, const double* v, double* o) {
    double t[3];
    for (int i = 0; i < 3; ++i) t[i] = a[3 * i] * v[0] + a[3 * i + 1] * v[1] + a[3 * i + 2] * v[2];
    memcpy(o, t, sizeof t);
}
static void hat3(const double* v, double* S) {
    S[0] = 0; S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2]; S[4] = 0; S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0]; S[8] = 0;
}
static double det3(const double* a) {
    return a[0] * (a[4] * a[8] - a[5] * a[7]) - a[1] * (a[3] * a[8] - a[5] * a[6]) + a[2] * (a[3] * a[7] - a[4] * a[6]);
}
static double norm3(const double* v) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

/* symmetric 3x3 eigen-decomposition by cyclic Jacobi: A = V diag(w) V^T */
static void sym3_eig(const double* A_in, double* w, double* V) {
    double A[9];
    memcpy(A, A_in, sizeof A);
    for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = A[1] * A[1] + A[2] * A[2] + A[5] * A[5];
        double dia = A[0] * A[0] + A[4] * A[4] + A[8] * A[8];
        if (off <= 1e-36 * dia || off == 0.0) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                double apq = A[3 * p + q];
                if (apq == 0.0) continue;
                double app = A[3 * p + p], aqq = A[3 * q + q];
                double theta = (aqq - app) / (2.0 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 3; ++k) { /* A = J^T A J */
                    double akp = A[3 * k + p], akq = A[3 * k + q];
                    A[3 * k + p] = c * akp - s * akq;
                    A[3 * k + q] = s * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {
                    double apk = A[3 * p + k], aqk = A[3 * q + k];
                    A[3 * p + k] = c * apk - s * aqk;
                    A[3 * q + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 3; ++k) {
                    double vkp = V[3 * k + p], vkq = V[3 * k + q];
                    V[3 * k + p] = c * vkp - s * vkq;
                    V[3 * k + q] = s * vkp + c * vkq;
                }
            }
    }
    w[0] = A[0]; w[1] = A[4]; w[2] = A[8];
}

/*
 * Nearest proper rotation of a 3x3 matrix: R = U diag(1,1,d) V^T with d = sign(det(U V^T)).
 * This is exactly what SO3d(const Matrix3d&) (LieUtils.cpp:275-288, U col 2 flipped when
 * det<0) and EstimateRotation (FeatureTracker.cpp:341-352, V col 2 flipped) compute; the result
 * is unique whenever the two largest singular values are distinct from the smallest.
 */
void oracle_nearest_rotation(const double* A, double* R) {
    double AtA[9], At[9], w[3], V[9];
    m3_tr(A, At);
    m3_mul(At, A, AtA);
    sym3_eig(AtA, w, V);
    /* sort eigenpairs descending */
    int idx[3] = {0, 1, 2};
    for (int i = 0; i < 3; ++i)
        for (int j = i + 1; j < 3; ++j)
            if (w[idx[j]] > w[idx[i]]) { int t = idx[i]; idx[i] = idx[j]; idx[j] = t; }
    double v[3][3], u[3][3];
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) v[c][r] = V[3 * r + idx[c]];
    for (int c = 0; c < 2; ++c) {
        m3_vec(A, v[c], u[c]);
        double n = norm3(u[c]);
        if (n > 0) { u[c][0] /= n; u[c][1] /= n; u[c][2] /= n; }
    }
    /* re-orthogonalise u1 against u0 (robust for near-degenerate input) */
    double d01 = u[0][0] * u[1][0] + u[0][1] * u[1][1] + u[0][2] * u[1][2];
    for (int r = 0; r < 3; ++r) u[1][r] -= d01 * u[0][r];
    double n1 = norm3(u[1]);
    if (n1 > 0) { u[1][0] /= n1; u[1][1] /= n1; u[1][2] /= n1; }
    u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
    u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
    u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
    double detV = det3(V); /* +-1; columns of V permuted => sign folds in below */
    double vm[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) vm[3 * r + c] = v[c][r];
    detV = det3(vm);
    /* det(U V^T) with u2 = u0 x u1 (det U = +1) equals det(V); choose d so det(R) = +1 */
    double d = (detV < 0) ? -1.0 : 1.0;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) R[3 * r + c] = u[0][r] * v[0][c] + u[1][r] * v[1][c] + d * u[2][r] * v[2][c];
}

/* SO3d::Exp (LieUtils.cpp:203-219) — result re-projected like every SO3d construction */
static void so3_exp(const double* w, double* R) {
    double th = norm3(w);
    double M[9];
    if (th < EPS_D) {
        hat3(w, M);
        M[0] += 1; M[4] += 1; M[8] += 1;
    } else {
        double k[3] = {w[0] / th, w[1] / th, w[2] / th}, K[9], K2[9];
        hat3(k, K);
        m3_mul(K, K, K2);
        double s = sin(th), c = 1.0 - cos(th);
        for (int i = 0; i < 9; ++i) M[i] = s * K[i] + c * K2[i];
        M[0] += 1; M[4] += 1; M[8] += 1;
    }
    oracle_nearest_rotation(M, R);
}

/* SE3d::exp (LieUtils.cpp:305-333), xi = [rho, phi] */
static void se3_exp(const double* xi, double* R, double* t) {
    const double* rho = xi;
    const double* phi = xi + 3;
    so3_exp(phi, R);
    double th = norm3(phi);
    if (th < EPS_D) {
        t[0] = rho[0]; t[1] = rho[1]; t[2] = rho[2];
    } else {
        double P[9], P2[9], Vm[9];
        hat3(phi, P);
        m3_mul(P, P, P2);
        double th2 = th * th, a = (1.0 - cos(th)) / th2, b = (th - sin(th)) / (th2 * th);
        for (int i = 0; i < 9; ++i) Vm[i] = a * P[i] + b * P2[i];
        Vm[0] += 1; Vm[4] += 1; Vm[8] += 1;
        m3_vec(Vm, rho, t);
    }
}

/* SE3d composition (LieUtils.h:268-271): (R1,t1)*(R2,t2), rotation re-projected */
static void se3_mul(const double* R1, const double* t1, const double* R2, const double* t2, double* R, double* t) {
    double M[9], tt[3];
    m3_mul(R1, R2, M);
    m3_vec(R1, t2, tt);
    tt[0] += t1[0]; tt[1] += t1[1]; tt[2] += t1[2];
    oracle_nearest_rotation(M, R);
    memcpy(t, tt, sizeof tt);
}
/* SE3d::inverse (LieUtils.h:279-282) */
static void se3_inv(const double* R, const double* t, double* Ri, double* ti) {
    double Rt[9], nt[3] = {-t[0], -t[1], -t[2]};
    m3_tr(R, Rt);
    oracle_nearest_rotation(Rt, Ri);
    m3_vec(Ri, nt, ti);
}

/* SO3 log as used by InertialFactorFixedGravity::log_SO3 (Factors.cpp:1507-1519) */
static void imu_log_so3(const double* R, double* w) {
    double tr = R[0] + R[4] + R[8];
    double c = (tr - 1.0) / 2.0;
    c = fmax(-1.0, fmin(1.0, c));
    double th = acos(c);
    double v[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};
    if (th < 1e-6) {
        w[0] = v[0] / 2.0; w[1] = v[1] / 2.0; w[2] = v[2] / 2.0;
        return;
    }
    double f = th / (2.0 * sin(th));
    w[0] = f * v[0]; w[1] = f * v[1]; w[2] = f * v[2];
}
/* InertialFactorFixedGravity::right_jacobian_SO3 (Factors.cpp:1495-1505) */
static void imu_right_jac(const double* phi, double* J) {
    double th = norm3(phi);
    if (th < 1e-6) {
        for (int i = 0; i < 9; ++i) J[i] = (i % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    double P[9], P2[9];
    hat3(phi, P);
    m3_mul(P, P, P2);
    double th2 = th * th, a = (1.0 - cos(th)) / th2, b = (th - sin(th)) / (th2 * th);
    for (int i = 0; i < 9; ++i) J[i] = -a * P[i] + b * P2[i];
    J[0] += 1; J[4] += 1; J[8] += 1;
}
/* plain SO3d::exp of a bias correction (SO3d::Exp, LieUtils.cpp:203-219) */
static void so3_exp_plain(const double* w, double* R) { so3_exp(w, R); }

/* general dense inverse by Gauss-Jordan with partial pivoting (Eigen .inverse() for 9x9) */
static int dense_inverse(int n, const double* A, double* Ai) {
    double* M = (double*)malloc(sizeof(double) * n * 2 * n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < 2 * n; ++j) M[i * 2 * n + j] = j < n ? A[i * n + j] : (j - n == i ? 1.0 : 0.0);
    for (int c = 0; c < n; ++c) {
        int p = c;
        for (int r = c + 1; r < n; ++r)
            if (fabs(M[r * 2 * n + c]) > fabs(M[p * 2 * n + c])) p = r;
        if (M[p * 2 * n + c] == 0.0) { free(M); return -1; }
        if (p != c)
            for (int j = 0; j < 2 * n; ++j) { double t = M[c * 2 * n + j]; M[c * 2 * n + j] = M[p * 2 * n + j]; M[p * 2 * n + j] = t; }
        double iv = 1.0 / M[c * 2 * n + c];
        for (int j = 0; j < 2 * n; ++j) M[c * 2 * n + j] *= iv;
        for (int r = 0; r < n; ++r) {
            if (r == c) continue;
            double f = M[r * 2 * n + c];
            if (f == 0.0) continue;
            for (int j = 0; j < 2 * n; ++j) M[r * 2 * n + j] -= f * M[c * 2 * n + j];
        }
    }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) Ai[i * n + j] = M[i * 2 * n + n + j];
    free(M);
    return 0;
}
/* in-place lower Cholesky of a dense SPD matrix (row-major, full storage); 0 on success */
static int dense_llt(int n, double* A) {
    for (int j = 0; j < n; ++j) {
        double d = A[j * n + j];
        for (int k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
        if (!(d > 0.0)) return -1;
        d = sqrt(d);
        A[j * n + j] = d;
        for (int i = j + 1; i < n; ++i) {
            double s = A[i * n + j];
            for (int k = 0; k < j; ++k) s -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = s / d;
        }
    }
    return 0;
}
static void dense_llt_solve(int n, const double* L, double* b) {
    for (int i = 0; i < n; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s -= L[i * n + k] * b[k];
        b[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = b[i];
        for (int k = i + 1; k < n; ++k) s -= L[k * n + i] * b[k];
        b[i] = s / L[i * n + i];
    }
}

/* ========================================================================================= */
/* Huber loss + Corrector                                                                     */
/* ========================================================================================= */
void oracle_huber(double delta, double s, double rho[3]) {
    double b = delta * delta, a = delta;
    if (s > b) {
        double r = sqrt(s);
        rho[0] = 2.0 * a * r - b;
        rho[1] = fmax(DBL_MIN, a / r);
        rho[2] = -rho[1] / (2.0 * s);
    } else {
        rho[0] = s; rho[1] = 1.0; rho[2] = 0.0;
    }
}
/* Corrector: residual_scaling and alpha_sq_norm (corrector.cc:42-98) */
void oracle_corrector(double sq_norm, const double rho[3], double* residual_scaling, double* alpha_sq_norm,
                      double* sqrt_rho1) {
    *sqrt_rho1 = sqrt(rho[1]);
    if (sq_norm == 0.0 || rho[2] <= 0.0) {
        *residual_scaling = *sqrt_rho1;
        *alpha_sq_norm = 0.0;
        return;
    }
    double D = 1.0 + 2.0 * sq_norm * rho[2] / rho[1];
    double alpha = 1.0 - sqrt(D);
    *residual_scaling = *sqrt_rho1 / (1 - alpha);
    *alpha_sq_norm = alpha / sq_norm;
}

/* ========================================================================================= */
/* Factors                                                                                    */
/* ========================================================================================= */
typedef struct {
    double R_init[9], t_init[3]; /* SE3d(T_wb_init): SVD-projected */
    double R_cb[9], t_cb[3];     /* SE3d(T_cb): SVD-projected */
    double R_cb_raw[9];          /* m_Tcb.block<3,3> used verbatim in the Jacobians */
} pose_ctx;

/*
 * BAFactor::Evaluate (Factors.cpp:327-542) / PnPFactor::Evaluate (:33-210).
 * Returns 1 on success, 0 when the PnP variant fails (L<1e-10 → Evaluate returns false).
 * r: weighted residual; Jp (2x6, row-major) and Jl (2x3) if non-NULL.
 */
static int factor_eval(const pose_ctx* pc, const double* delta, const double* Pw, double u_obs, double v_obs,
                       double cols, double rows, const double* Lw /* chol(info) lower 2x2 or NULL */, int outlier,
                       int is_pnp, double* r, double* Jp, double* Jl) {
    if (outlier) {
        r[0] = 640.0; r[1] = 480.0;
        if (Jp) memset(Jp, 0, 12 * sizeof(double));
        if (Jl) memset(Jl, 0, 6 * sizeof(double));
        return 1;
    }
    double dR[9], dt[3], Rwb[9], twb[3], Rbw[9], tbw[3], Rcw[9], tcw[3];
    se3_exp(delta, dR, dt);
    se3_mul(pc->R_init, pc->t_init, dR, dt, Rwb, twb);
    se3_inv(Rwb, twb, Rbw, tbw);
    se3_mul(pc->R_cb, pc->t_cb, Rbw, tbw, Rcw, tcw);
    double Pc[3];
    m3_vec(Rcw, Pw, Pc);
    Pc[0] += tcw[0]; Pc[1] += tcw[1]; Pc[2] += tcw[2];
    double x = Pc[0], y = Pc[1], z = Pc[2];
    double L = norm3(Pc);
    if (L < 1e-10) {
        if (Jp) memset(Jp, 0, 12 * sizeof(double));
        if (Jl) memset(Jl, 0, 6 * sizeof(double));
        if (is_pnp) return 0;
        r[0] = 640.0; r[1] = 360.0;
        return 1;
    }
    double theta = atan2(x, z);
    double phi = -asin(y / L);
    double u = cols * (0.5 + theta / (2.0 * M_PI));
    double v = rows * (0.5 - phi / M_PI);
    double du = u_obs - u, dv = v_obs - v;
    if (du > cols / 2.0) du -= cols;
    else if (du < -cols / 2.0) du += cols;
    if (fabs(du) > 100.0 || fabs(dv) > 100.0) {
        r[0] = 100.0; r[1] = 100.0;
        if (Jp) memset(Jp, 0, 12 * sizeof(double));
        if (Jl) memset(Jl, 0, 6 * sizeof(double));
        return 1;
    }
    if (Lw) {
        r[0] = Lw[0] * du;
        r[1] = Lw[2] * du + Lw[3] * dv;
    } else {
        r[0] = du; r[1] = dv;
    }
    if (!Jp && !Jl) return 1;
    double xz2 = x * x + z * z, L2 = L * L, xzn = sqrt(xz2);
    if (xz2 < 1e-10 || L2 < 1e-10) {
        if (Jp) memset(Jp, 0, 12 * sizeof(double));
        if (Jl) memset(Jl, 0, 6 * sizeof(double));
        return 1;
    }
    double Jc[6];
    Jc[0] = -cols / (2.0 * M_PI) * z / xz2;
    Jc[1] = 0.0;
    Jc[2] = cols / (2.0 * M_PI) * x / xz2;
    Jc[3] = rows / M_PI * (x * y) / (L2 * xzn);
    Jc[4] = -rows / M_PI * xzn / L2;
    Jc[5] = rows / M_PI * (y * z) / (L2 * xzn);
    double Jw[6];
    if (Lw) {
        for (int j = 0; j < 3; ++j) {
            Jw[j] = Lw[0] * Jc[j];
            Jw[3 + j] = Lw[2] * Jc[j] + Lw[3] * Jc[3 + j];
        }
    } else {
        memcpy(Jw, Jc, sizeof Jw);
    }
    if (Jp) {
        double Pb[3], H[9], RH[9];
        m3_vec(Rbw, Pw, Pb);
        Pb[0] += tbw[0]; Pb[1] += tbw[1]; Pb[2] += tbw[2];
        hat3(Pb, H);
        m3_mul(pc->R_cb_raw, H, RH);
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 3; ++j) {
                double st = 0, sr = 0;
                for (int k = 0; k < 3; ++k) {
                    st += Jw[3 * i + k] * (-pc->R_cb_raw[3 * k + j]);
                    sr += Jw[3 * i + k] * RH[3 * k + j];
                }
                Jp[6 * i + j] = st;
                Jp[6 * i + 3 + j] = sr;
            }
    }
    if (Jl) {
        double Cp[9];
        m3_mul(pc->R_cb_raw, Rbw, Cp);
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 3; ++j) {
                double s = 0;
                for (int k = 0; k < 3; ++k) s += Jw[3 * i + k] * Cp[3 * k + j];
                Jl[3 * i + j] = s;
            }
    }
    return 1;
}

/* BAFactor::compute_chi_square (Factors.cpp:544-612); PnP variant (:212-265) ignores the flag */
static double factor_chi2(const pose_ctx* pc, const double* delta, const double* Pw, double u_obs, double v_obs,
                          double cols, double rows, const double* info, int outlier, int is_pnp) {
    if (outlier && !is_pnp) return 0.0;
    double dR[9], dt[3], Rwb[9], twb[3], Rbw[9], tbw[3], Rcw[9], tcw[3];
    se3_exp(delta, dR, dt);
    se3_mul(pc->R_init, pc->t_init, dR, dt, Rwb, twb);
    se3_inv(Rwb, twb, Rbw, tbw);
    se3_mul(pc->R_cb, pc->t_cb, Rbw, tbw, Rcw, tcw);
    double Pc[3];
    m3_vec(Rcw, Pw, Pc);
    Pc[0] += tcw[0]; Pc[1] += tcw[1]; Pc[2] += tcw[2];
    double L = norm3(Pc);
    if (L < 1e-10) return is_pnp ? DBL_MAX : 1000.0;
    double theta = atan2(Pc[0], Pc[2]);
    double phi = -asin(Pc[1] / L);
    double u = cols * (0.5 + theta / (2.0 * M_PI));
    double v = rows * (0.5 - phi / M_PI);
    double du = u_obs - u, dv = v_obs - v;
    if (du > cols / 2.0) du -= cols;
    else if (du < -cols / 2.0) du += cols;
    return du * (info[0] * du + info[1] * dv) + dv * (info[2] * du + info[3] * dv);
}

/* InertialFactorFixedGravity (Factors.cpp:1299-1485) */
typedef struct {
    double sqrt_info[81];
    double dR[9], dV[3], dP[3], JRg[9], JVg[9], JVa[9], JPg[9], JPa[9], bg0[3], ba0[3];
    double dt;
    double Ri_init[9], ti_init[3], Rj_init[9], tj_init[3];
    double g[3];
} imu_ctx;

static void imu_ctx_init(imu_ctx* c, const vio_preint* p, const double* g, const vio_pose* Ti, const vio_pose* Tj) {
    double cov[81], info[81];
    for (int i = 0; i < 81; ++i) cov[i] = (double)p->cov9[i];
    for (int i = 0; i < 9; ++i) cov[i * 9 + i] += 1e-8;
    int ok = dense_inverse(9, cov, info) == 0;
    if (ok) ok = dense_llt(9, info) == 0; /* info now holds L (lower) + stale upper */
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 9; ++j) c->sqrt_info[i * 9 + j] = ok ? (j >= i ? info[j * 9 + i] : 0.0) : (i == j ? 1.0 : 0.0);
    for (int i = 0; i < 9; ++i) {
        c->dR[i] = p->delta_R[i]; c->JRg[i] = p->J_Rg[i]; c->JVg[i] = p->J_Vg[i];
        c->JVa[i] = p->J_Va[i]; c->JPg[i] = p->J_Pg[i]; c->JPa[i] = p->J_Pa[i];
    }
    for (int i = 0; i < 3; ++i) {
        c->dV[i] = p->delta_V[i]; c->dP[i] = p->delta_P[i];
        c->bg0[i] = p->gyro_bias[i]; c->ba0[i] = p->accel_bias[i]; c->g[i] = g[i];
    }
    c->dt = p->dt_total;
    oracle_nearest_rotation(Ti->R, c->Ri_init);
    memcpy(c->ti_init, Ti->t, sizeof c->ti_init);
    oracle_nearest_rotation(Tj->R, c->Rj_init);
    memcpy(c->tj_init, Tj->t, sizeof c->tj_init);
}

/* r[9]; J_vi/J_bg/J_ba/J_vj 9x3 row-major (pose Jacobians are identically zero, :1415-1419) */
static void imu_eval(const imu_ctx* c, const double* di, const double* vi, const double* bg, const double* ba,
                     const double* dj, const double* vj, double* r, double* Jvi, double* Jbg, double* Jba,
                     double* Jvj) {
    double dR[9], dt3[3], Rwi[9], twi[3], Rwj[9], twj[3], Rbwi[9];
    se3_exp(di, dR, dt3);
    se3_mul(c->Ri_init, c->ti_init, dR, dt3, Rwi, twi);
    se3_exp(dj, dR, dt3);
    se3_mul(c->Rj_init, c->tj_init, dR, dt3, Rwj, twj);
    m3_tr(Rwi, Rbwi);
    double dt = c->dt;
    double DR[9], DV[3], DP[3];
    memcpy(DR, c->dR, sizeof DR);
    memcpy(DV, c->dV, sizeof DV);
    memcpy(DP, c->dP, sizeof DP);
    double dbg[3] = {bg[0] - c->bg0[0], bg[1] - c->bg0[1], bg[2] - c->bg0[2]};
    double dba[3] = {ba[0] - c->ba0[0], ba[1] - c->ba0[1], ba[2] - c->ba0[2]};
    if (norm3(dbg) > 1e-6 || norm3(dba) > 1e-6) {
        double w[3], E[9], t1[3], t2[3];
        m3_vec(c->JRg, dbg, w);
        so3_exp_plain(w, E);
        m3_mul(DR, E, DR); /* plain Matrix3d product: delta_R is not an SO3d (Factors.cpp:1381) */
        m3_vec(c->JVg, dbg, t1); m3_vec(c->JVa, dba, t2);
        for (int i = 0; i < 3; ++i) DV[i] += t1[i] + t2[i];
        m3_vec(c->JPg, dbg, t1); m3_vec(c->JPa, dba, t2);
        for (int i = 0; i < 3; ++i) DP[i] += t1[i] + t2[i];
    }
    double raw[9];
    {
        double DRt[9], A[9], B[9];
        m3_tr(DR, DRt);
        m3_mul(DRt, Rbwi, A);
        m3_mul(A, Rwj, B);
        imu_log_so3(B, raw);
        double tv[3], ev[3];
        for (int i = 0; i < 3; ++i) tv[i] = vj[i] - vi[i] - c->g[i] * dt;
        m3_vec(Rbwi, tv, ev);
        for (int i = 0; i < 3; ++i) raw[3 + i] = ev[i] - DV[i];
        for (int i = 0; i < 3; ++i) tv[i] = twj[i] - twi[i] - vi[i] * dt - 0.5 * c->g[i] * dt * dt;
        m3_vec(Rbwi, tv, ev);
        for (int i = 0; i < 3; ++i) raw[6 + i] = ev[i] - DP[i];
    }
    for (int i = 0; i < 9; ++i) {
        double s = 0;
        for (int k = 0; k < 9; ++k) s += c->sqrt_info[i * 9 + k] * raw[k];
        r[i] = s;
    }
    if (!Jvi) return;
    const double* S = c->sqrt_info;
    /* J_vi: rows 3..5 = -S33(3,3) R_bwi ; rows 6..8 = -S(6,6) R_bwi dt */
    memset(Jvi, 0, 27 * sizeof(double));
    memset(Jvj, 0, 27 * sizeof(double));
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double a = 0, b = 0;
            for (int k = 0; k < 3; ++k) {
                a += S[(3 + i) * 9 + 3 + k] * Rbwi[3 * k + j];
                b += S[(6 + i) * 9 + 6 + k] * Rbwi[3 * k + j];
            }
            Jvi[(3 + i) * 3 + j] = -a;
            Jvi[(6 + i) * 3 + j] = -b * dt;
            Jvj[(3 + i) * 3 + j] = a;
        }
    /* J_bg = S * [-Jr^{-1}(-er) J_Rg ; -J_Vg ; -J_Pg]  with er the WEIGHTED rotation residual */
    double mer[3] = {-r[0], -r[1], -r[2]}, Jr[9], Jri[9], T[27], A[9];
    imu_right_jac(mer, Jr);
    dense_inverse(3, Jr, Jri);
    m3_mul(Jri, c->JRg, A);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            T[i * 3 + j] = -A[3 * i + j];
            T[(3 + i) * 3 + j] = -c->JVg[3 * i + j];
            T[(6 + i) * 3 + j] = -c->JPg[3 * i + j];
        }
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int k = 0; k < 9; ++k) s += S[i * 9 + k] * T[k * 3 + j];
            Jbg[i * 3 + j] = s;
        }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            T[i * 3 + j] = 0.0;
            T[(3 + i) * 3 + j] = -c->JVa[3 * i + j];
            T[(6 + i) * 3 + j] = -c->JPa[3 * i + j];
        }
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int k = 0; k < 9; ++k) s += S[i * 9 + k] * T[k * 3 + j];
            Jba[i * 3 + j] = s;
        }
}

/* exported single-factor evaluators for golden/FD tests */
static void pose_ctx_init_(pose_ctx* pc, const vio_pose* Twb, const vio_pose* Tcb) {
    oracle_nearest_rotation(Twb->R, pc->R_init);
    memcpy(pc->t_init, Twb->t, sizeof pc->t_init);
    oracle_nearest_rotation(Tcb->R, pc->R_cb);
    memcpy(pc->t_cb, Tcb->t, sizeof pc->t_cb);
    memcpy(pc->R_cb_raw, Tcb->R, sizeof pc->R_cb_raw);
}
int oracle_ba_factor(const vio_pose* T_wb_init, const vio_pose* T_cb, const double* delta, const double* Pw,
                     double u, double v, double cols, double rows, int outlier, int is_pnp, double* r,
                     double* Jp, double* Jl) {
    pose_ctx pc;
    oracle_nearest_rotation(T_wb_init->R, pc.R_init);
    memcpy(pc.t_init, T_wb_init->t, sizeof pc.t_init);
    oracle_nearest_rotation(T_cb->R, pc.R_cb);
    memcpy(pc.t_cb, T_cb->t, sizeof pc.t_cb);
    memcpy(pc.R_cb_raw, T_cb->R, sizeof pc.R_cb_raw);
    return factor_eval(&pc, delta, Pw, u, v, cols, rows, NULL, outlier, is_pnp, r, Jp, Jl);
}
double oracle_ba_chi2(const vio_pose* T_wb_init, const vio_pose* T_cb, const double* delta, const double* Pw,
                      double u, double v, double cols, double rows, int outlier, int is_pnp) {
    pose_ctx pc;
    pose_ctx_init_(&pc, T_wb_init, T_cb);
    const double info[4] = {1.0, 0.0, 0.0, 1.0};
    return factor_chi2(&pc, delta, Pw, u, v, cols, rows, info, outlier, is_pnp);
}
void oracle_imu_factor(const vio_preint* p, const double* g, const vio_pose* Ti, const vio_pose* Tj,
                       const double* di, const double* vi, const double* bg, const double* ba, const double* dj,
                       const double* vj, double* r, double* Jvi, double* Jbg, double* Jba, double* Jvj,
                       double* sqrt_info) {
    imu_ctx c;
    imu_ctx_init(&c, p, g, Ti, Tj);
    imu_eval(&c, di, vi, bg, ba, dj, vj, r, Jvi, Jbg, Jba, Jvj);
    if (sqrt_info) memcpy(sqrt_info, c.sqrt_info, sizeof c.sqrt_info);
}

/* ========================================================================================= */
/* Block-sparse Schur complement (Ceres SchurEliminator::Eliminate / BackSubstitute,           */
/* internal/ceres/schur_eliminator_impl.h:179-377; DENSE/SPARSE_SCHUR's reduced system,        */
/* schur_complement_solver.cc:118-176).  Generic over block sizes: the BA step (ba_solve) and   */
/* the restated Ceres fixtures (LinearLeastSquaresProblem2/4 with schur_eliminator_test.cc)     */
/* run the same code.                                                                         */
/* ========================================================================================= */
typedef struct {
    int n_cols;             /* column blocks */
    const int* col_size;    /* scalar size of each column block */
    const int* col_pos;     /* position of the block in the full solution vector x */
    const int* col_red;     /* f-blocks: position in the reduced system; e-blocks: -1 */
    int n_red;              /* reduced system size */
    int n_rows;             /* row blocks (residual blocks) */
    const int* row_size;
    const int* row_pos;     /* position of the row block in b */
    const int* row_cell;    /* CSR: cells of row r are row_cell[r] .. row_cell[r+1]-1 */
    const int* cell_col;    /* column block of the cell (at most one e-block per row) */
    const int* cell_off;    /* row-major row_size x col_size values of the cell in `values` */
    const double* values;
} oracle_bsm;

static int bsm_is_e(const oracle_bsm* A, int cb) { return A->col_red[cb] < 0; }

/* small dense kernels of the eliminator: C (m x n, leading dim ldc) += A^T B with A rs x m, B rs x n
   (row-major); out (m) += A^T b.  The common BA shapes are dispatched with constant sizes so the
   compiler unrolls them (a generic loop nest is ~3x slower, and this oracle is also the CPU baseline). */
static inline __attribute__((always_inline)) void k_tn(int rs, int m, int n, const double* A, const double* B,
                                                       double* C, size_t ldc, double sign) {
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) {
            double acc = 0.0;
            for (int t = 0; t < rs; ++t) acc += A[t * m + i] * B[t * n + j];
            C[i * ldc + j] += sign * acc;
        }
}
static void acc_tn(int rs, int m, int n, const double* A, const double* B, double* C, size_t ldc) {
    if (rs == 2 && m == 6 && n == 6) k_tn(2, 6, 6, A, B, C, ldc, 1.0);
    else if (rs == 2 && m == 6 && n == 3) k_tn(2, 6, 3, A, B, C, ldc, 1.0);
    else if (rs == 2 && m == 3 && n == 3) k_tn(2, 3, 3, A, B, C, ldc, 1.0);
    else if (rs == 9 && m == 3 && n == 3) k_tn(9, 3, 3, A, B, C, ldc, 1.0);
    else k_tn(rs, m, n, A, B, C, ldc, 1.0);
}
static inline __attribute__((always_inline)) void k_tv(int rs, int m, const double* A, const double* b, double* out) {
    for (int i = 0; i < m; ++i) {
        double acc = 0.0;
        for (int t = 0; t < rs; ++t) acc += A[t * m + i] * b[t];
        out[i] += acc;
    }
}
static void acc_tv(int rs, int m, const double* A, const double* b, double* out) {
    if (rs == 2 && m == 6) k_tv(2, 6, A, b, out);
    else if (rs == 2 && m == 3) k_tv(2, 3, A, b, out);
    else if (rs == 9 && m == 3) k_tv(9, 3, A, b, out);
    else k_tv(rs, m, A, b, out);
}
/* C (m x n, ldc) -= Y Z^T with Y m x es, Z n x es (Z rows with leading dim es) */
static inline __attribute__((always_inline)) void k_ytz(int m, int n, int es, const double* Y, const double* Z,
                                                        double* C, size_t ldc) {
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) {
            double acc = 0.0;
            for (int t = 0; t < es; ++t) acc += Y[i * es + t] * Z[j * es + t];
            C[i * ldc + j] -= acc;
        }
}
static void sub_ytz(int m, int n, int es, const double* Y, const double* Z, double* C, size_t ldc) {
    if (m == 6 && n == 6 && es == 3) k_ytz(6, 6, 3, Y, Z, C, ldc);
    else if (m == 3 && n == 3 && es == 3) k_ytz(3, 3, 3, Y, Z, C, ldc);
    else if (m == 6 && n == 3 && es == 3) k_ytz(6, 3, 3, Y, Z, C, ldc);
    else if (m == 3 && n == 6 && es == 3) k_ytz(3, 6, 3, Y, Z, C, ldc);
    else k_ytz(m, n, es, Y, Z, C, ldc);
}

/* E^T E + diag(D_e)^2 of e-block e over its rows, inverted by LLT (schur_eliminator_impl.h:226-240,
   BlockRandomAccessDiagonalMatrix::Invert); Einv is es x es. rows: the e-block's row list. */
static int bsm_e_inverse(const oracle_bsm* A, int e, const int* rows, int nr, const double* D, double* Einv) {
    const int es = A->col_size[e];
    double M[9 * 9];
    memset(M, 0, sizeof(double) * es * es);
    for (int q = 0; q < nr; ++q) {
        const int r = rows[q], rs = A->row_size[r];
        for (int c = A->row_cell[r]; c < A->row_cell[r + 1]; ++c) {
            if (A->cell_col[c] != e) continue;
            const double* E = A->values + A->cell_off[c];
            acc_tn(rs, es, es, E, E, M, es);
        }
    }
    if (D)
        for (int i = 0; i < es; ++i) M[i * es + i] += D[A->col_pos[e] + i] * D[A->col_pos[e] + i];
    if (dense_llt(es, M) != 0) return 0;
    for (int c = 0; c < es; ++c) {
        double v[9] = {0};
        v[c] = 1.0;
        dense_llt_solve(es, M, v);
        for (int r = 0; r < es; ++r) Einv[r * es + c] = v[r];
    }
    return 1;
}

/* row lists per e-block (rows without an e-cell go to the list n_e == "f-only") */
static int* bsm_row_groups(const oracle_bsm* A, int** ptr_out) {
    int* ecell = (int*)malloc(sizeof(int) * (A->n_rows > 0 ? A->n_rows : 1));
    int* ptr = (int*)calloc(A->n_cols + 2, sizeof(int));
    for (int r = 0; r < A->n_rows; ++r) {
        int e = A->n_cols; /* sentinel: no e-block */
        for (int c = A->row_cell[r]; c < A->row_cell[r + 1]; ++c)
            if (bsm_is_e(A, A->cell_col[c])) e = A->cell_col[c];
        ecell[r] = e;
        ptr[e + 1]++;
    }
    for (int e = 0; e <= A->n_cols; ++e) ptr[e + 1] += ptr[e];
    int* list = (int*)malloc(sizeof(int) * (A->n_rows > 0 ? A->n_rows : 1));
    int* fill = (int*)calloc(A->n_cols + 1, sizeof(int));
    for (int r = 0; r < A->n_rows; ++r) list[ptr[ecell[r]] + fill[ecell[r]]++] = r;
    free(fill); free(ecell);
    *ptr_out = ptr;
    return list;
}

/* lhs (n_red x n_red, full symmetric, row-major) = F^T F + D_f^2 - F^T E (E^T E + D_e^2)^-1 E^T F,
   rhs = F^T b - F^T E (E^T E + D_e^2)^-1 E^T b.  D may be NULL (no regularisation).  Returns 0 if an
   e-block is not positive definite. */
static int schur_eliminate_mt(const oracle_bsm* A, const double* b, const double* D, double* lhs, double* rhs);

int oracle_schur_eliminate(const oracle_bsm* A, const double* b, const double* D, double* lhs, double* rhs) {
    const int S = A->n_red;
    if (oracle_threads > 1 && S <= 1024) return schur_eliminate_mt(A, b, D, lhs, rhs);
    memset(lhs, 0, sizeof(double) * (size_t)S * S);
    memset(rhs, 0, sizeof(double) * S);
    if (D)
        for (int cb = 0; cb < A->n_cols; ++cb) {
            if (bsm_is_e(A, cb)) continue;
            for (int i = 0; i < A->col_size[cb]; ++i)
                lhs[(size_t)(A->col_red[cb] + i) * S + A->col_red[cb] + i] += D[A->col_pos[cb] + i] * D[A->col_pos[cb] + i];
        }
    int* ptr;
    int* list = bsm_row_groups(A, &ptr);
    /* F^T F and F^T b of every row (schur_eliminator_impl.h:384-420 ChunkOuterProduct / NoEBlockRowsUpdate) */
    for (int r = 0; r < A->n_rows; ++r) {
        const int rs = A->row_size[r];
        const double* br = b + A->row_pos[r];
        for (int c1 = A->row_cell[r]; c1 < A->row_cell[r + 1]; ++c1) {
            const int f1 = A->cell_col[c1];
            if (bsm_is_e(A, f1)) continue;
            const int s1 = A->col_size[f1], o1 = A->col_red[f1];
            const double* F1 = A->values + A->cell_off[c1];
            acc_tv(rs, s1, F1, br, rhs + o1);
            for (int c2 = A->row_cell[r]; c2 < A->row_cell[r + 1]; ++c2) {
                const int f2 = A->cell_col[c2];
                if (bsm_is_e(A, f2)) continue;
                const int s2 = A->col_size[f2], o2 = A->col_red[f2];
                const double* F2 = A->values + A->cell_off[c2];
                acc_tn(rs, s1, s2, F1, F2, lhs + (size_t)o1 * S + o2, S);
            }
        }
    }
    /* per e-block chunk: Y_f = (F^T E)_f Einv, lhs -= Y_f1 (F^T E)_f2^T, rhs -= Y_f E^T b */
    int ok = 1;
    double* FtE = (double*)malloc(sizeof(double) * (size_t)(S > 0 ? S : 1) * 9);
    uint8_t* touched = (uint8_t*)calloc(A->n_cols > 0 ? A->n_cols : 1, 1);
    int* tlist = (int*)malloc(sizeof(int) * (A->n_cols > 0 ? A->n_cols : 1));
    for (int e = 0; e < A->n_cols && ok; ++e) {
        if (!bsm_is_e(A, e)) continue;
        const int* rows = list + ptr[e];
        const int nr = ptr[e + 1] - ptr[e];
        const int es = A->col_size[e];
        double Einv[81], Etb[9] = {0};
        if (!bsm_e_inverse(A, e, rows, nr, D, Einv)) { ok = 0; break; }
        /* the f-blocks sharing a row with e (first-seen order), their F^T E rows zeroed */
        int nt = 0;
        for (int q = 0; q < nr; ++q)
            for (int c = A->row_cell[rows[q]]; c < A->row_cell[rows[q] + 1]; ++c) {
                const int f = A->cell_col[c];
                if (bsm_is_e(A, f) || touched[f]) continue;
                touched[f] = 1;
                tlist[nt++] = f;
                memset(FtE + (size_t)A->col_red[f] * es, 0, sizeof(double) * A->col_size[f] * es);
            }
        for (int q = 0; q < nr; ++q) {
            const int r = rows[q], rs = A->row_size[r];
            const double* E = NULL;
            for (int c = A->row_cell[r]; c < A->row_cell[r + 1]; ++c)
                if (A->cell_col[c] == e) E = A->values + A->cell_off[c];
            const double* br = b + A->row_pos[r];
            acc_tv(rs, es, E, br, Etb);
            for (int c = A->row_cell[r]; c < A->row_cell[r + 1]; ++c) {
                const int f = A->cell_col[c];
                if (bsm_is_e(A, f)) continue;
                const int fs = A->col_size[f], of = A->col_red[f];
                acc_tn(rs, fs, es, A->values + A->cell_off[c], E, FtE + (size_t)of * es, es);
            }
        }
        for (int a = 0; a < nt; ++a) {
            const int f1 = tlist[a];
            const int s1 = A->col_size[f1], o1 = A->col_red[f1];
            double Y[9 * 9];  /* Y = (F^T E)_f1 Einv, s1 x es */
            for (int i = 0; i < s1; ++i) {
                for (int j = 0; j < es; ++j) {
                    double acc = 0.0;
                    for (int t = 0; t < es; ++t) acc += FtE[(size_t)(o1 + i) * es + t] * Einv[t * es + j];
                    Y[i * es + j] = acc;
                }
                double acc = 0.0;
                for (int j = 0; j < es; ++j) acc += Y[i * es + j] * Etb[j];
                rhs[o1 + i] -= acc;
            }
            for (int bq = 0; bq < nt; ++bq) {
                const int f2 = tlist[bq];
                sub_ytz(s1, A->col_size[f2], es, Y, FtE + (size_t)A->col_red[f2] * es, lhs + (size_t)o1 * S + A->col_red[f2], S);
            }
        }
        for (int a = 0; a < nt; ++a) touched[tlist[a]] = 0;
    }
    free(FtE); free(touched); free(tlist); free(list); free(ptr);
    return ok;
}

/* The same elimination with the e-block chunks spread over oracle_threads threads (Ceres'
   ParallelFor over chunks, schur_eliminator_impl.h:179-260): each thread accumulates its chunks'
   updates into a private reduced system, the partials are added in thread order. */
static int schur_eliminate_mt(const oracle_bsm* A, const double* b, const double* D, double* lhs, double* rhs) {
    const int S = A->n_red, T = oracle_threads;
    memset(lhs, 0, sizeof(double) * (size_t)S * S);
    memset(rhs, 0, sizeof(double) * S);
    if (D)
        for (int cb = 0; cb < A->n_cols; ++cb) {
            if (bsm_is_e(A, cb)) continue;
            for (int i = 0; i < A->col_size[cb]; ++i)
                lhs[(size_t)(A->col_red[cb] + i) * S + A->col_red[cb] + i] += D[A->col_pos[cb] + i] * D[A->col_pos[cb] + i];
        }
    int* ptr;
    int* list = bsm_row_groups(A, &ptr);
    for (int r = 0; r < A->n_rows; ++r) {
        const int rs = A->row_size[r];
        const double* br = b + A->row_pos[r];
        for (int c1 = A->row_cell[r]; c1 < A->row_cell[r + 1]; ++c1) {
            const int f1 = A->cell_col[c1];
            if (bsm_is_e(A, f1)) continue;
            const int s1 = A->col_size[f1], o1 = A->col_red[f1];
            const double* F1 = A->values + A->cell_off[c1];
            acc_tv(rs, s1, F1, br, rhs + o1);
            for (int c2 = A->row_cell[r]; c2 < A->row_cell[r + 1]; ++c2) {
                const int f2 = A->cell_col[c2];
                if (bsm_is_e(A, f2)) continue;
                acc_tn(rs, s1, A->col_size[f2], F1, A->values + A->cell_off[c2], lhs + (size_t)o1 * S + A->col_red[f2], S);
            }
        }
    }
    const size_t SS = (size_t)(S > 0 ? S : 1);
    double* part = (double*)calloc((size_t)T * (SS * SS + SS), sizeof(double));
    int ok = 1;
#pragma omp parallel num_threads(T) reduction(&& : ok)
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        double* pl = part + (size_t)tid * (SS * SS + SS);
        double* pr = pl + SS * SS;
        double* FtE = (double*)malloc(sizeof(double) * SS * 9);
        uint8_t* touched = (uint8_t*)calloc(A->n_cols > 0 ? A->n_cols : 1, 1);
        int* tlist = (int*)malloc(sizeof(int) * (A->n_cols > 0 ? A->n_cols : 1));
#pragma omp for schedule(static)
        for (int e = 0; e < A->n_cols; ++e) {
            if (!bsm_is_e(A, e) || !ok) continue;
            const int* rows = list + ptr[e];
            const int nr = ptr[e + 1] - ptr[e];
            const int es = A->col_size[e];
            double Einv[81], Etb[9] = {0};
            if (!bsm_e_inverse(A, e, rows, nr, D, Einv)) { ok = 0; continue; }
            int nt = 0;
            for (int q = 0; q < nr; ++q)
                for (int c = A->row_cell[rows[q]]; c < A->row_cell[rows[q] + 1]; ++c) {
                    const int f = A->cell_col[c];
                    if (bsm_is_e(A, f) || touched[f]) continue;
                    touched[f] = 1;
                    tlist[nt++] = f;
                    memset(FtE + (size_t)A->col_red[f] * es, 0, sizeof(double) * A->col_size[f] * es);
                }
            for (int q = 0; q < nr; ++q) {
                const int r = rows[q], rs = A->row_size[r];
                const double* E = NULL;
                for (int c = A->row_cell[r]; c < A->row_cell[r + 1]; ++c)
                    if (A->cell_col[c] == e) E = A->values + A->cell_off[c];
                acc_tv(rs, es, E, b + A->row_pos[r], Etb);
                for (int c = A->row_cell[r]; c < A->row_cell[r + 1]; ++c) {
                    const int f = A->cell_col[c];
                    if (bsm_is_e(A, f)) continue;
                    acc_tn(rs, A->col_size[f], es, A->values + A->cell_off[c], E, FtE + (size_t)A->col_red[f] * es, es);
                }
            }
            for (int a = 0; a < nt; ++a) {
                const int f1 = tlist[a];
                const int s1 = A->col_size[f1], o1 = A->col_red[f1];
                double Y[9 * 9];
                for (int i = 0; i < s1; ++i) {
                    for (int j = 0; j < es; ++j) {
                        double acc = 0.0;
                        for (int t = 0; t < es; ++t) acc += FtE[(size_t)(o1 + i) * es + t] * Einv[t * es + j];
                        Y[i * es + j] = acc;
                    }
                    double acc = 0.0;
                    for (int j = 0; j < es; ++j) acc += Y[i * es + j] * Etb[j];
                    pr[o1 + i] -= acc;
                }
                for (int bq = 0; bq < nt; ++bq) {
                    const int f2 = tlist[bq];
                    sub_ytz(s1, A->col_size[f2], es, Y, FtE + (size_t)A->col_red[f2] * es, pl + (size_t)o1 * S + A->col_red[f2], S);
                }
            }
            for (int a = 0; a < nt; ++a) touched[tlist[a]] = 0;
        }
        free(FtE); free(touched); free(tlist);
    }
    for (int t = 0; t < T; ++t) {
        const double* pl = part + (size_t)t * (SS * SS + SS);
        for (size_t i = 0; i < (size_t)S * S; ++i) lhs[i] += pl[i];
        for (int i = 0; i < S; ++i) rhs[i] += pl[SS * SS + i];
    }
    free(part); free(list); free(ptr);
    return ok;
}

/* x (full vector): f-blocks copied from z (reduced solution), e-blocks
   x_e = (E^T E + D_e^2)^-1 E^T (b - sum_f F z_f) (schur_eliminator_impl.h:311-377) */
int oracle_schur_back_substitute(const oracle_bsm* A, const double* b, const double* D, const double* z, double* x) {
    for (int cb = 0; cb < A->n_cols; ++cb)
        if (!bsm_is_e(A, cb))
            for (int i = 0; i < A->col_size[cb]; ++i) x[A->col_pos[cb] + i] = z[A->col_red[cb] + i];
    int* ptr;
    int* list = bsm_row_groups(A, &ptr);
    int ok = 1;
    /* the e-blocks are independent: threads only change which core computes each one */
#pragma omp parallel for num_threads(oracle_threads) schedule(static) reduction(&& : ok) if (oracle_threads > 1)
    for (int e = 0; e < A->n_cols; ++e) {
        if (!bsm_is_e(A, e) || !ok) continue;
        const int* rows = list + ptr[e];
        const int nr = ptr[e + 1] - ptr[e];
        const int es = A->col_size[e];
        double Einv[81], rhs[9] = {0};
        if (!bsm_e_inverse(A, e, rows, nr, D, Einv)) { ok = 0; continue; }
        for (int q = 0; q < nr; ++q) {
            const int r = rows[q], rs = A->row_size[r];
            double sres[9];
            const double* E = NULL;
            for (int t = 0; t < rs; ++t) sres[t] = b[A->row_pos[r] + t];
            for (int c = A->row_cell[r]; c < A->row_cell[r + 1]; ++c) {
                const int f = A->cell_col[c];
                if (f == e) { E = A->values + A->cell_off[c]; continue; }
                const int fs = A->col_size[f];
                const double* F = A->values + A->cell_off[c];
                for (int t = 0; t < rs; ++t) {
                    double acc = 0.0;
                    for (int i = 0; i < fs; ++i) acc += F[t * fs + i] * z[A->col_red[f] + i];
                    sres[t] -= acc;
                }
            }
            for (int i = 0; i < es; ++i)
                for (int t = 0; t < rs; ++t) rhs[i] += E[t * es + i] * sres[t];
        }
        for (int i = 0; i < es; ++i) {
            double acc = 0.0;
            for (int j = 0; j < es; ++j) acc += Einv[i * es + j] * rhs[j];
            x[A->col_pos[e] + i] = acc;
        }
    }
    free(list); free(ptr);
    return ok;
}

/* SchurComplementSolver::SolveImpl (schur_complement_solver.cc:118-176): eliminate, dense LLT of the
   reduced system (an empty one when every column block is eliminated), back-substitute.  x: full
   solution of min |A x - b|^2 + |D x|^2 (D may be NULL).  Returns 0 on a non-positive-definite block. */
int oracle_schur_solve(const oracle_bsm* A, const double* b, const double* D, double* x) {
    const int S = A->n_red;
    double* lhs = (double*)malloc(sizeof(double) * (size_t)(S > 0 ? S : 1) * (S > 0 ? S : 1));
    double* rhs = (double*)malloc(sizeof(double) * (S > 0 ? S : 1));
    int ok = oracle_schur_eliminate(A, b, D, lhs, rhs);
    if (ok && S > 0) {
        if (dense_llt(S, lhs) != 0) ok = 0;
        else dense_llt_solve(S, lhs, rhs);
    }
    if (ok) ok = oracle_schur_back_substitute(A, b, D, rhs, x);
    free(lhs); free(rhs);
    return ok;
}

/* ========================================================================================= */
/* Generic Ceres-2.0 LM minimiser (TrustRegionMinimizer + LevenbergMarquardtStrategy)         */
/* ========================================================================================= */
typedef struct {
    int n;
    void* user;
    /* evaluate at x; cost out; when want_jac, cache Jacobian + residuals internally and write the
       unscaled gradient J^T r into g and squared column norms into colsq. Return 1 ok, 0 fail. */
    int (*eval)(void* user, const double* x, double* cost, int want_jac, double* g, double* colsq);
    /* solve (J~^T J~ + D^2) y = J~^T r with J~ = J diag(s); return 1 ok, 0 linear-solver failure */
    int (*solve)(void* user, const double* s, const double* D, double* y);
    /* model cost change -(J~ h)^T (r + J~ h / 2) for the scaled step h */
    double (*model_change)(void* user, const double* s, const double* h);
} lm_problem;

typedef struct {
    int max_iterations;
    int fixed_iterations; /* disable all convergence tests */
    double function_tolerance, gradient_tolerance, parameter_tolerance;
    double initial_radius, max_radius, min_radius, min_relative_decrease;
    double min_diagonal, max_diagonal;
    int max_consecutive_invalid;
    double fixed_cost;
} lm_options;

typedef struct {
    int termination;
    int iterations; /* iterations.size() */
    int successful, unsuccessful;
    double initial_cost, final_cost;
    /* Solver::Summary::iterations (tests compare it with the HIP path's trace) */
    int trace_n;
    vio_ba_iteration trace[256];
} lm_summary;

void oracle_lm_default_options(lm_options* o) {
    o->max_iterations = 50;
    o->fixed_iterations = 0;
    o->function_tolerance = 1e-6;
    o->gradient_tolerance = 1e-10;
    o->parameter_tolerance = 1e-8;
    o->initial_radius = 1e4;
    o->max_radius = 1e16;
    o->min_radius = 1e-32;
    o->min_relative_decrease = 1e-3;
    o->min_diagonal = 1e-6;
    o->max_diagonal = 1e32;
    o->max_consecutive_invalid = 5;
    o->fixed_cost = 0.0;
}

/* LevenbergMarquardtStrategy radius updates (levenberg_marquardt_strategy.cc:147-160) */
typedef struct { double radius, decrease_factor, max_radius; } lm_radius;
void oracle_lm_step_accepted(lm_radius* s, double q) {
    s->radius = s->radius / fmax(1.0 / 3.0, 1.0 - pow(2.0 * q - 1.0, 3));
    s->radius = fmin(s->max_radius, s->radius);
    s->decrease_factor = 2.0;
}
void oracle_lm_step_rejected(lm_radius* s) {
    s->radius = s->radius / s->decrease_factor;
    s->decrease_factor *= 2.0;
}

/* FinalizeIterationAndCheckIfMinimizerCanContinue pushes the iteration summary (trust_region_minimizer.cc:313-348) */
static void push_trace(lm_summary* sum, const vio_ba_iteration* it, double radius) {
    if (sum->trace_n < 256) {
        sum->trace[sum->trace_n] = *it;
        sum->trace[sum->trace_n].trust_region_radius = radius;
        sum->trace_n++;
    }
}

/* gradient_max_norm = |x - Plus(x, -g)|_inf (trust_region_minimizer.cc:288-299; Plus is x + delta:
   no local parameterization is registered), which differs from |g|_inf by the roundoff of x - g */
static double grad_max_norm(int n, const double* x, const double* g) {
    double m = 0.0;
    for (int i = 0; i < n; ++i) m = fmax(m, fabs(x[i] - (x[i] + (-g[i]))));
    return m;
}

/* LM diagonal D = sqrt(clamp(diag(J~^T J~), min, max) / radius) (levenberg_marquardt_strategy.cc:76-88),
   with diag(J~^T J~) = colsq .* s .* s for the Jacobi-scaled Jacobian */
void oracle_lm_diagonal(int n, const double* colsq, const double* s, double radius, double dmin, double dmax,
                        double* D) {
    for (int i = 0; i < n; ++i) {
        double d = colsq[i] * s[i] * s[i];
        d = fmin(fmax(d, dmin), dmax);
        D[i] = sqrt(d / radius);
    }
}

/* x in/out: on return holds the solution Ceres would copy back to the user */
/* wall time of each LM iteration of the calling thread's last minimisation (ComputeTrustRegionStep
   through the step's acceptance / re-linearisation): the CPU baseline of a single iteration without the
   set-up and IterationZero of the solve (bench.py, config 5) */
static __thread double g_iter_sec[64];
static __thread int g_iter_n;
static double now_sec(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
int oracle_iter_seconds(double* out, int cap) {
    const int n = g_iter_n < cap ? g_iter_n : cap;
    for (int i = 0; i < n; ++i) out[i] = g_iter_sec[i];
    return g_iter_n;
}

int oracle_lm_minimize(const lm_problem* P, const lm_options* opt, double* x_user, lm_summary* sum) {
    const int n = P->n;
    memset(sum, 0, sizeof *sum);
    sum->termination = VIO_TERM_NO_CONVERGENCE;
    double* x = (double*)malloc(sizeof(double) * n);
    double* x0 = (double*)malloc(sizeof(double) * n);
    double* g = (double*)malloc(sizeof(double) * n);
    double* colsq = (double*)malloc(sizeof(double) * n);
    double* s = (double*)malloc(sizeof(double) * n);
    double* D = (double*)malloc(sizeof(double) * n);
    double* y = (double*)malloc(sizeof(double) * n);
    double* delta = (double*)malloc(sizeof(double) * n);
    double* cand = (double*)malloc(sizeof(double) * n);
    memcpy(x, x_user, sizeof(double) * n);
    memcpy(x0, x_user, sizeof(double) * n);
    double x_norm = -1.0; /* trust_region_minimizer.cc:185 */
    double x_cost = DBL_MAX;
    double minimum_cost = DBL_MAX;
    lm_radius rad = {opt->initial_radius, 2.0, opt->max_radius};
    int consecutive_invalid = 0;
    const int fixed = opt->fixed_iterations;

    /* IterationZero */
    if (!P->eval(P->user, x, &x_cost, 1, g, colsq)) {
        sum->termination = VIO_TERM_FAILURE;
        sum->initial_cost = opt->fixed_cost; /* never set by Ceres on this path */
        sum->final_cost = sum->initial_cost;
        goto done;
    }
    for (int i = 0; i < n; ++i) s[i] = 1.0 / (1.0 + sqrt(colsq[i]));
    double gmax = grad_max_norm(n, x, g);
    sum->initial_cost = x_cost + opt->fixed_cost;
    vio_ba_iteration it; /* IterationZero (:195-229) */
    memset(&it, 0, sizeof it);
    it.step_is_valid = it.step_is_successful = 1;
    it.cost = x_cost + opt->fixed_cost;
    it.gradient_max_norm = gmax;
    double step_evaluator_current = x_cost;
    int iteration = 0;
    int step_successful = 1;
    double iter_cost = x_cost + opt->fixed_cost;
    double final_cost = sum->initial_cost;
    double model_change = 0, cand_cost = 0;

    g_iter_n = 0;
    double t_iter = -1.0;
    for (;;) {
        if (t_iter >= 0.0 && g_iter_n < 64) g_iter_sec[g_iter_n++] = now_sec() - t_iter;
        /* FinalizeIterationAndCheckIfMinimizerCanContinue */
        if (step_successful) {
            sum->successful++;
            if (x_cost < minimum_cost) {
                minimum_cost = x_cost;
                memcpy(x_user, x, sizeof(double) * n);
            }
        } else {
            sum->unsuccessful++;
        }
        sum->iterations++;
        final_cost = fmin(final_cost, iter_cost);
        push_trace(sum, &it, rad.radius);
        if (iteration >= opt->max_iterations) { sum->termination = VIO_TERM_NO_CONVERGENCE; break; }
        if (!fixed && step_successful && gmax <= opt->gradient_tolerance) { sum->termination = VIO_TERM_CONVERGENCE; break; }
        if (!fixed && rad.radius <= opt->min_radius) { sum->termination = VIO_TERM_CONVERGENCE; break; }

        iteration++;
        t_iter = now_sec();
        memset(&it, 0, sizeof it);
        it.iteration = iteration;
        /* ComputeTrustRegionStep */
        oracle_lm_diagonal(n, colsq, s, rad.radius, opt->min_diagonal, opt->max_diagonal, D);
        int valid = P->solve(P->user, s, D, y);
        if (valid) {
            for (int i = 0; i < n; ++i)
                if (!isfinite(y[i])) valid = 0;
        }
        model_change = 0.0;
        if (valid) {
            for (int i = 0; i < n; ++i) y[i] = -y[i]; /* trust_region_step */
            model_change = P->model_change(P->user, s, y);
            valid = model_change > 0.0;
        }
        it.model_cost_change = model_change;
        if (!valid) {
            /* HandleInvalidStep (:453-486): a zero-length, no-progress iteration */
            if (++consecutive_invalid >= opt->max_consecutive_invalid) {
                sum->termination = VIO_TERM_FAILURE;
                break;
            }
            oracle_lm_step_rejected(&rad);
            step_successful = 0;
            iter_cost = x_cost + opt->fixed_cost;
            it.cost = iter_cost;
            it.gradient_max_norm = gmax;
            continue;
        }
        it.step_is_valid = 1;
        consecutive_invalid = 0;
        for (int i = 0; i < n; ++i) delta[i] = y[i] * s[i];
        for (int i = 0; i < n; ++i) cand[i] = x[i] + delta[i];
        if (!P->eval(P->user, cand, &cand_cost, 0, NULL, NULL)) cand_cost = DBL_MAX;

        /* ParameterToleranceReached */
        double step_norm = 0;
        for (int i = 0; i < n; ++i) { double d = x[i] - cand[i]; step_norm += d * d; }
        step_norm = sqrt(step_norm);
        it.step_norm = step_norm;
        it.cost_change = x_cost - cand_cost;
        if (!fixed && step_norm <= opt->parameter_tolerance * (x_norm + opt->parameter_tolerance)) {
            sum->termination = VIO_TERM_CONVERGENCE;
            break;
        }
        /* FunctionToleranceReached */
        if (!fixed && fabs(x_cost - cand_cost) <= opt->function_tolerance * x_cost) {
            sum->termination = VIO_TERM_CONVERGENCE;
            break;
        }
        /* IsStepSuccessful */
        double rel;
        if (cand_cost >= DBL_MAX) rel = -DBL_MAX;
        else rel = (step_evaluator_current - cand_cost) / model_change;
        it.relative_decrease = rel;
        if (rel > opt->min_relative_decrease) {
            /* HandleSuccessfulStep */
            memcpy(x, cand, sizeof(double) * n);
            double xn = 0;
            for (int i = 0; i < n; ++i) xn += x[i] * x[i];
            x_norm = sqrt(xn);
            if (!P->eval(P->user, x, &x_cost, 1, g, colsq)) {
                sum->termination = VIO_TERM_FAILURE;
                break;
            }
            gmax = grad_max_norm(n, x, g);
            step_successful = 1;
            oracle_lm_step_accepted(&rad, rel);
            step_evaluator_current = cand_cost;
            iter_cost = x_cost + opt->fixed_cost;
        } else {
            step_successful = 0;
            iter_cost = cand_cost + opt->fixed_cost;
            oracle_lm_step_rejected(&rad);
        }
        it.step_is_successful = step_successful;
        it.cost = iter_cost;
        it.gradient_max_norm = gmax; /* kept from the last successful step when rejected (:118-129) */
    }
    sum->final_cost = final_cost;
done:
    if (sum->termination == VIO_TERM_FAILURE) memcpy(x_user, x0, sizeof(double) * n);
    free(x); free(x0); free(g); free(colsq); free(s); free(D); free(y); free(delta); free(cand);
    return 0;
}

/* ========================================================================================= */
/* BA problem on top of the generic minimiser                                                 */
/* ========================================================================================= */
typedef struct {
    const vio_ba_problem* p;
    int K, L, N;
    int is_pnp, is_vi;
    pose_ctx* pc;       /* K */
    double Lw[4];       /* chol(info) lower */
    double info[4];
    /* parameter layout */
    int* pose_off;      /* K: offset into x or -1 (constant or unused) */
    int* lm_off;        /* L: offset (e-block) or -1 */
    int* vel_off;       /* K */
    int bg_off, ba_off;
    int nf;             /* number of f-parameters (poses, velocities, biases) */
    int n;              /* total */
    int* f_index;       /* map f-param global offset -> 0..nf-1 (size n, -1 for points) */
    /* current values of every block (constant ones included) */
    double* pose_val;   /* K*6 */
    double* lm_val;     /* L*3 */
    double* vel_val;    /* K*3 */
    double bg_val[3], ba_val[3];
    /* residual blocks */
    uint8_t* obs_active; /* N */
    uint8_t* obs_outlier;/* N (PnP rounds) */
    imu_ctx* imu;        /* K (entry k links k-1 -> k) */
    uint8_t* imu_active; /* K */
    /* cached linearisation */
    double* r;           /* N*2 corrected residuals */
    double* Jp;          /* N*12 */
    double* Jl;          /* N*6 */
    double* ri;          /* K*9 */
    double* Ji;          /* K*4*27 (vi, bg, ba, vj) */
    /* CSR of observations per landmark */
    int* lm_ptr;
    int* lm_obs;
    int eval_failed;
    /* the scaled Jacobian as a block-sparse matrix for the Schur eliminator (built once) */
    oracle_bsm A;
    int *col_size, *col_pos, *col_red, *row_size, *row_pos, *row_cell, *cell_col, *cell_off;
    int* cell_src;       /* per cell: observation o (pose cell: 2*o, point cell: 2*o+1) or IMU block -(1 + 4k + b) */
    double* values;
    double* bvec;        /* residuals in row order */
    int* row_src;        /* per row: observation o, or -(1 + k) for the IMU factor k-1 -> k */
    /* per-observation scratch of the multi-threaded evaluation (oracle_threads > 1) */
    double* obs_tmp;     /* N */
    uint8_t* obs_ok;     /* N */
} ba_ctx;

static void ba_unpack(ba_ctx* c, const double* x) {
    for (int k = 0; k < c->K; ++k) {
        if (c->pose_off[k] >= 0) memcpy(c->pose_val + 6 * k, x + c->pose_off[k], 6 * sizeof(double));
        if (c->vel_off && c->vel_off[k] >= 0) memcpy(c->vel_val + 3 * k, x + c->vel_off[k], 3 * sizeof(double));
    }
    for (int l = 0; l < c->L; ++l)
        if (c->lm_off[l] >= 0) memcpy(c->lm_val + 3 * l, x + c->lm_off[l], 3 * sizeof(double));
    if (c->bg_off >= 0) memcpy(c->bg_val, x + c->bg_off, 3 * sizeof(double));
    if (c->ba_off >= 0) memcpy(c->ba_val, x + c->ba_off, 3 * sizeof(double));
}

/* evaluate one visual residual block with the loss applied; returns 0 on factor failure */
static int ba_eval_obs(ba_ctx* c, int o, double* cost, double* r, double* Jp, double* Jl) {
    const vio_ba_problem* p = c->p;
    int k = p->obs_kf[o], l = p->obs_lm[o];
    double rr[2];
    int ok = factor_eval(&c->pc[k], c->pose_val + 6 * k, c->lm_val + 3 * l, (double)p->obs_uv[2 * o],
                         (double)p->obs_uv[2 * o + 1], p->cols, p->rows, c->Lw, c->obs_outlier[o], c->is_pnp, rr, Jp, Jl);
    if (!ok) return 0;
    double sq = rr[0] * rr[0] + rr[1] * rr[1], rho[3];
    oracle_huber(p->huber_delta, sq, rho);
    *cost = 0.5 * rho[0];
    double rs, asq, sr1;
    oracle_corrector(sq, rho, &rs, &asq, &sr1);
    if (Jp || Jl) {
        /* CorrectJacobian uses the UNcorrected residual (residual_block.cc:178-189) */
        double* Js[2] = {Jp, Jl};
        int nc[2] = {6, 3};
        for (int b = 0; b < 2; ++b) {
            double* J = Js[b];
            if (!J) continue;
            if (asq == 0.0) {
                for (int i = 0; i < 2 * nc[b]; ++i) J[i] *= sr1;
            } else {
                for (int cc = 0; cc < nc[b]; ++cc) {
                    double rtj = J[cc] * rr[0] + J[nc[b] + cc] * rr[1];
                    for (int row = 0; row < 2; ++row)
                        J[row * nc[b] + cc] = sr1 * (J[row * nc[b] + cc] - asq * rr[row] * rtj);
                }
            }
        }
    }
    r[0] = rr[0] * rs;
    r[1] = rr[1] * rs;
    return 1;
}

static int ba_eval(void* user, const double* x, double* cost, int want_jac, double* g, double* colsq) {
    ba_ctx* c = (ba_ctx*)user;
    ba_unpack(c, x);
    double total = 0.0;
    if (want_jac) {
        memset(g, 0, sizeof(double) * c->n);
        memset(colsq, 0, sizeof(double) * c->n);
    }
    /* multi-threaded: the factors are evaluated in parallel first, the sums below keep their order */
    const int mt = oracle_threads > 1;
    if (mt) {
#pragma omp parallel for num_threads(oracle_threads) schedule(static)
        for (int o = 0; o < c->N; ++o) {
            if (!c->obs_active[o]) continue;
            double r[2];
            c->obs_ok[o] = (uint8_t)ba_eval_obs(c, o, &c->obs_tmp[o], r, want_jac ? c->Jp + 12 * o : NULL,
                                                want_jac ? c->Jl + 6 * o : NULL);
            if (want_jac) {
                c->r[2 * o] = r[0];
                c->r[2 * o + 1] = r[1];
            }
        }
    }
    for (int o = 0; o < c->N; ++o) {
        if (!c->obs_active[o]) continue;
        int k = c->p->obs_kf[o], l = c->p->obs_lm[o];
        double cst, r[2];
        double* Jp = want_jac ? c->Jp + 12 * o : NULL;
        double* Jl = want_jac ? c->Jl + 6 * o : NULL;
        if (mt) {
            if (!c->obs_ok[o]) return 0;
            cst = c->obs_tmp[o];
            if (want_jac) { r[0] = c->r[2 * o]; r[1] = c->r[2 * o + 1]; }
        } else if (!ba_eval_obs(c, o, &cst, r, Jp, Jl)) {
            return 0;
        }
        total += cst;
        if (want_jac) {
            c->r[2 * o] = r[0];
            c->r[2 * o + 1] = r[1];
            int po = c->pose_off[k], lo = c->lm_off[l];
            if (po >= 0)
                for (int j = 0; j < 6; ++j) {
                    g[po + j] += Jp[j] * r[0] + Jp[6 + j] * r[1];
                    colsq[po + j] += Jp[j] * Jp[j] + Jp[6 + j] * Jp[6 + j];
                }
            if (lo >= 0)
                for (int j = 0; j < 3; ++j) {
                    g[lo + j] += Jl[j] * r[0] + Jl[3 + j] * r[1];
                    colsq[lo + j] += Jl[j] * Jl[j] + Jl[3 + j] * Jl[3 + j];
                }
        }
    }
    if (c->is_vi) {
        for (int k = 1; k < c->K; ++k) {
            if (!c->imu_active[k]) continue;
            double r[9];
            double* J = c->Ji + 108 * k;
            imu_eval(&c->imu[k], c->pose_val + 6 * (k - 1), c->vel_val + 3 * (k - 1), c->bg_val, c->ba_val,
                     c->pose_val + 6 * k, c->vel_val + 3 * k, r, want_jac ? J : NULL, want_jac ? J + 27 : NULL,
                     want_jac ? J + 54 : NULL, want_jac ? J + 81 : NULL);
            double sq = 0;
            for (int i = 0; i < 9; ++i) sq += r[i] * r[i];
            total += 0.5 * sq;
            if (want_jac) {
                memcpy(c->ri + 9 * k, r, sizeof r);
                int offs[4] = {c->vel_off[k - 1], c->bg_off, c->ba_off, c->vel_off[k]};
                for (int b = 0; b < 4; ++b) {
                    if (offs[b] < 0) continue;
                    for (int j = 0; j < 3; ++j)
                        for (int i = 0; i < 9; ++i) {
                            double v = J[27 * b + 3 * i + j];
                            g[offs[b] + j] += v * r[i];
                            colsq[offs[b] + j] += v * v;
                        }
                }
            }
        }
    }
    *cost = total;
    return 1;
}

/* Schur complement solve: points are the e-blocks, everything else the reduced system.  The scaled
   Jacobian J~ = J diag(s) goes through the generic eliminator (oracle_schur_eliminate, pinned by the
   Ceres SchurEliminatorTest fixtures), the reduced system through a dense LLT (SPARSE_SCHUR's LDLT is
   the same factorisation up to roundoff), the points through oracle_schur_back_substitute. */
static int ba_solve(void* user, const double* s, const double* D, double* y) {
    ba_ctx* c = (ba_ctx*)user;
    const oracle_bsm* A = &c->A;
    /* values of J~ and the residual vector, row by row */
#pragma omp parallel for num_threads(oracle_threads) schedule(static) if (oracle_threads > 1)
    for (int r = 0; r < A->n_rows; ++r) {
        const int src = c->row_src[r];
        if (src >= 0) {
            c->bvec[A->row_pos[r]] = c->r[2 * src];
            c->bvec[A->row_pos[r] + 1] = c->r[2 * src + 1];
        } else {
            memcpy(c->bvec + A->row_pos[r], c->ri + 9 * (-src - 1), 9 * sizeof(double));
        }
        for (int q = A->row_cell[r]; q < A->row_cell[r + 1]; ++q) {
            const int cs = c->cell_src[q], cb = A->cell_col[q], w = A->col_size[cb], pos = A->col_pos[cb];
            double* v = c->values + A->cell_off[q];
            if (cs >= 0) {
                const int o = cs >> 1;
                const double* J = (cs & 1) ? c->Jl + 6 * o : c->Jp + 12 * o;
                for (int t = 0; t < 2; ++t)
                    for (int j = 0; j < w; ++j) v[t * w + j] = J[t * w + j] * s[pos + j];
            } else {
                const int k = (-cs - 1) >> 2, b = (-cs - 1) & 3;
                const double* J = c->Ji + 108 * k + 27 * b;
                for (int t = 0; t < 9; ++t)
                    for (int j = 0; j < 3; ++j) v[3 * t + j] = J[3 * t + j] * s[pos + j];
            }
        }
    }
    return oracle_schur_solve(A, c->bvec, D, y);
}

static double ba_model_change(void* user, const double* s, const double* h) {
    ba_ctx* c = (ba_ctx*)user;
    const vio_ba_problem* p = c->p;
    double mc = 0.0;
    /* per-observation terms (in parallel when oracle_threads > 1), summed in observation order */
#pragma omp parallel for num_threads(oracle_threads) schedule(static) if (oracle_threads > 1)
    for (int o = 0; o < c->N; ++o) {
        if (!c->obs_active[o]) continue;
        int po = c->pose_off[p->obs_kf[o]], lo = c->lm_off[p->obs_lm[o]];
        double m[2] = {0, 0};
        if (po >= 0)
            for (int j = 0; j < 6; ++j) {
                double hj = s[po + j] * h[po + j];
                m[0] += c->Jp[12 * o + j] * hj;
                m[1] += c->Jp[12 * o + 6 + j] * hj;
            }
        if (lo >= 0)
            for (int j = 0; j < 3; ++j) {
                double hj = s[lo + j] * h[lo + j];
                m[0] += c->Jl[6 * o + j] * hj;
                m[1] += c->Jl[6 * o + 3 + j] * hj;
            }
        c->obs_tmp[o] = m[0] * (c->r[2 * o] + m[0] / 2.0) + m[1] * (c->r[2 * o + 1] + m[1] / 2.0);
    }
    for (int o = 0; o < c->N; ++o)
        if (c->obs_active[o]) mc -= c->obs_tmp[o];
    if (c->is_vi) {
        for (int k = 1; k < c->K; ++k) {
            if (!c->imu_active[k]) continue;
            const double* J = c->Ji + 108 * k;
            int offs[4] = {c->vel_off[k - 1], c->bg_off, c->ba_off, c->vel_off[k]};
            double m[9] = {0};
            for (int b = 0; b < 4; ++b) {
                if (offs[b] < 0) continue;
                for (int i = 0; i < 9; ++i)
                    for (int j = 0; j < 3; ++j) m[i] += J[27 * b + 3 * i + j] * s[offs[b] + j] * h[offs[b] + j];
            }
            for (int i = 0; i < 9; ++i) mc -= m[i] * (c->ri[9 * k + i] + m[i] / 2.0);
        }
    }
    return mc;
}

/* ------------------------------------------------------------------------------------------ */
static void pose_ctx_init(pose_ctx* pc, const vio_pose* Twb, const vio_pose* Tcb) {
    oracle_nearest_rotation(Twb->R, pc->R_init);
    memcpy(pc->t_init, Twb->t, sizeof pc->t_init);
    oracle_nearest_rotation(Tcb->R, pc->R_cb);
    memcpy(pc->t_cb, Tcb->t, sizeof pc->t_cb);
    memcpy(pc->R_cb_raw, Tcb->R, sizeof pc->R_cb_raw);
}

/* column blocks: poses, velocities, biases (f-blocks at their x offsets, the reduced system's
   order), points (e-blocks); row blocks: active observations (2 rows: point and pose cells), then
   the IMU factors (9 rows: v_i, bg, ba, v_j cells) */
static void ba_build_bsm(ba_ctx* c) {
    const vio_ba_problem* p = c->p;
    const int K = c->K, L = c->L, N = c->N;
    int nc = 0;
    const int cap_c = 2 * K + 2 + L + 1;
    c->col_size = (int*)malloc(sizeof(int) * cap_c);
    c->col_pos = (int*)malloc(sizeof(int) * cap_c);
    c->col_red = (int*)malloc(sizeof(int) * cap_c);
    int* pose_cb = (int*)malloc(sizeof(int) * K);
    int* vel_cb = (int*)malloc(sizeof(int) * K);
    int* lm_cb = (int*)malloc(sizeof(int) * (L > 0 ? L : 1));
#define ADD_COL(sz, pos, red) (c->col_size[nc] = (sz), c->col_pos[nc] = (pos), c->col_red[nc] = (red), nc++)
    for (int k = 0; k < K; ++k) pose_cb[k] = c->pose_off[k] >= 0 ? ADD_COL(6, c->pose_off[k], c->pose_off[k]) : -1;
    for (int k = 0; k < K; ++k) vel_cb[k] = c->vel_off[k] >= 0 ? ADD_COL(3, c->vel_off[k], c->vel_off[k]) : -1;
    const int bg_cb = c->bg_off >= 0 ? ADD_COL(3, c->bg_off, c->bg_off) : -1;
    const int ba_cb = c->ba_off >= 0 ? ADD_COL(3, c->ba_off, c->ba_off) : -1;
    for (int l = 0; l < L; ++l) lm_cb[l] = c->lm_off[l] >= 0 ? ADD_COL(3, c->lm_off[l], -1) : -1;
#undef ADD_COL
    int nr = 0, ncell = 0, nval = 0, bpos = 0;
    const int cap_r = N + K + 1;
    c->row_size = (int*)malloc(sizeof(int) * cap_r);
    c->row_pos = (int*)malloc(sizeof(int) * cap_r);
    c->row_cell = (int*)malloc(sizeof(int) * (cap_r + 1));
    c->row_src = (int*)malloc(sizeof(int) * cap_r);
    c->cell_col = (int*)malloc(sizeof(int) * (2 * N + 4 * K + 1));
    c->cell_off = (int*)malloc(sizeof(int) * (2 * N + 4 * K + 1));
    c->cell_src = (int*)malloc(sizeof(int) * (2 * N + 4 * K + 1));
    c->row_cell[0] = 0;
    for (int o = 0; o < N; ++o) {
        if (!c->obs_active[o]) continue;
        const int pc_ = pose_cb[p->obs_kf[o]], lc = lm_cb[p->obs_lm[o]];
        c->row_size[nr] = 2; c->row_pos[nr] = bpos; c->row_src[nr] = o; bpos += 2;
        if (lc >= 0) { c->cell_col[ncell] = lc; c->cell_off[ncell] = nval; c->cell_src[ncell] = 2 * o + 1; ncell++; nval += 6; }
        if (pc_ >= 0) { c->cell_col[ncell] = pc_; c->cell_off[ncell] = nval; c->cell_src[ncell] = 2 * o; ncell++; nval += 12; }
        c->row_cell[++nr] = ncell;
    }
    if (c->is_vi)
        for (int k = 1; k < K; ++k) {
            if (!c->imu_active[k]) continue;
            c->row_size[nr] = 9; c->row_pos[nr] = bpos; c->row_src[nr] = -(1 + k); bpos += 9;
            const int cbs[4] = {vel_cb[k - 1], bg_cb, ba_cb, vel_cb[k]};
            for (int b = 0; b < 4; ++b) {
                if (cbs[b] < 0) continue;
                c->cell_col[ncell] = cbs[b]; c->cell_off[ncell] = nval; c->cell_src[ncell] = -(1 + 4 * k + b);
                ncell++; nval += 27;
            }
            c->row_cell[++nr] = ncell;
        }
    c->values = (double*)malloc(sizeof(double) * (nval > 0 ? nval : 1));
    c->bvec = (double*)malloc(sizeof(double) * (bpos > 0 ? bpos : 1));
    oracle_bsm A = {nc, c->col_size, c->col_pos, c->col_red, c->nf, nr, c->row_size, c->row_pos, c->row_cell,
                    c->cell_col, c->cell_off, c->values};
    c->A = A;
    free(pose_cb); free(vel_cb); free(lm_cb);
}

static int ba_ctx_build(ba_ctx* c, const vio_ba_problem* p) {
    memset(c, 0, sizeof *c);
    c->p = p;
    c->K = p->num_kf; c->L = p->num_lm; c->N = p->num_obs;
    c->is_pnp = p->variant == VIO_PNP;
    c->is_vi = p->variant == VIO_BA_VI;
    int K = c->K, L = c->L, N = c->N;
    c->pc = (pose_ctx*)malloc(sizeof(pose_ctx) * K);
    for (int k = 0; k < K; ++k) pose_ctx_init(&c->pc[k], &p->T_wb_init[k], &p->T_cb[k]);
    /* chol(info): identity info → L = I (Eigen LLT of the 2x2) */
    memcpy(c->info, p->info, sizeof c->info);
    {
        double a = p->info[0], b = p->info[2], d = p->info[3];
        if (a > 0) {
            double l00 = sqrt(a), l10 = b / l00, t = d - l10 * l10;
            if (t > 0) { c->Lw[0] = l00; c->Lw[1] = 0; c->Lw[2] = l10; c->Lw[3] = sqrt(t); }
            else { c->Lw[0] = 1; c->Lw[1] = 0; c->Lw[2] = 0; c->Lw[3] = 1; }
        } else { c->Lw[0] = 1; c->Lw[1] = 0; c->Lw[2] = 0; c->Lw[3] = 1; }
    }
    c->pose_val = (double*)calloc(6 * K, sizeof(double));
    c->lm_val = (double*)malloc(sizeof(double) * 3 * (L > 0 ? L : 1));
    memcpy(c->lm_val, p->lm_xyz, sizeof(double) * 3 * L);
    c->vel_val = (double*)calloc(3 * K, sizeof(double));
    if (c->is_vi) {
        memcpy(c->vel_val, p->vel, sizeof(double) * 3 * K);
        memcpy(c->bg_val, p->bg, sizeof c->bg_val);
        memcpy(c->ba_val, p->ba, sizeof c->ba_val);
    }
    c->obs_active = (uint8_t*)calloc(N > 0 ? N : 1, 1);
    c->obs_outlier = (uint8_t*)calloc(N > 0 ? N : 1, 1);
    c->r = (double*)calloc(2 * (size_t)(N > 0 ? N : 1), sizeof(double));
    c->Jp = (double*)calloc(12 * (size_t)(N > 0 ? N : 1), sizeof(double));
    c->Jl = (double*)calloc(6 * (size_t)(N > 0 ? N : 1), sizeof(double));
    c->obs_tmp = (double*)calloc(N > 0 ? N : 1, sizeof(double));
    c->obs_ok = (uint8_t*)calloc(N > 0 ? N : 1, 1);
    c->imu = (imu_ctx*)calloc(K, sizeof(imu_ctx));
    c->imu_active = (uint8_t*)calloc(K, 1);
    c->ri = (double*)calloc(9 * K, sizeof(double));
    c->Ji = (double*)calloc(108 * K, sizeof(double));
    /* which blocks are variable and used */
    uint8_t* pose_used = (uint8_t*)calloc(K, 1);
    uint8_t* lm_used = (uint8_t*)calloc(L > 0 ? L : 1, 1);
    uint8_t* vel_used = (uint8_t*)calloc(K, 1);
    int bias_used = 0;
    for (int o = 0; o < N; ++o) {
        int k = p->obs_kf[o], l = p->obs_lm[o];
        int kvar = !p->kf_const[k];
        int lvar = !c->is_pnp && !p->lm_const[l];
        if (kvar || lvar) {
            c->obs_active[o] = 1;
            if (kvar) pose_used[k] = 1;
            if (lvar) lm_used[l] = 1;
        }
    }
    if (c->is_vi) {
        for (int k = 1; k < K; ++k) {
            if (!p->preint_valid[k]) continue;
            c->imu_active[k] = 1; /* velocities and biases are never constant in RunVIBA */
            imu_ctx_init(&c->imu[k], &p->preint[k], p->gravity, &p->T_wb_init[k - 1], &p->T_wb_init[k]);
            vel_used[k - 1] = vel_used[k] = 1;
            bias_used = 1;
            /* pose blocks of an IMU factor enter the problem through it as well */
            if (!p->kf_const[k - 1]) pose_used[k - 1] = 1;
            if (!p->kf_const[k]) pose_used[k] = 1;
        }
    }
    c->pose_off = (int*)malloc(sizeof(int) * K);
    c->vel_off = (int*)malloc(sizeof(int) * K);
    c->lm_off = (int*)malloc(sizeof(int) * (L > 0 ? L : 1));
    int off = 0;
    for (int k = 0; k < K; ++k) { c->pose_off[k] = pose_used[k] ? off : -1; if (pose_used[k]) off += 6; }
    for (int k = 0; k < K; ++k) { c->vel_off[k] = vel_used[k] ? off : -1; if (vel_used[k]) off += 3; }
    c->bg_off = bias_used ? off : -1; if (bias_used) off += 3;
    c->ba_off = bias_used ? off : -1; if (bias_used) off += 3;
    c->nf = off;
    for (int l = 0; l < L; ++l) { c->lm_off[l] = lm_used[l] ? off : -1; if (lm_used[l]) off += 3; }
    c->n = off;
    c->f_index = (int*)malloc(sizeof(int) * (off > 0 ? off : 1));
    for (int i = 0; i < off; ++i) c->f_index[i] = i < c->nf ? i : -1;
    /* CSR by landmark */
    c->lm_ptr = (int*)calloc(L + 1, sizeof(int));
    c->lm_obs = (int*)malloc(sizeof(int) * (N > 0 ? N : 1));
    for (int o = 0; o < N; ++o) c->lm_ptr[p->obs_lm[o] + 1]++;
    for (int l = 0; l < L; ++l) c->lm_ptr[l + 1] += c->lm_ptr[l];
    int* fill = (int*)calloc(L > 0 ? L : 1, sizeof(int));
    for (int o = 0; o < N; ++o) {
        int l = p->obs_lm[o];
        c->lm_obs[c->lm_ptr[l] + fill[l]++] = o;
    }
    free(fill);
    free(pose_used); free(lm_used); free(vel_used);
    ba_build_bsm(c);
    return 0;
}

static void ba_ctx_free(ba_ctx* c) {
    free(c->pc); free(c->pose_val); free(c->lm_val); free(c->vel_val); free(c->obs_active); free(c->obs_outlier);
    free(c->r); free(c->Jp); free(c->Jl); free(c->imu); free(c->imu_active); free(c->ri); free(c->Ji);
    free(c->pose_off); free(c->vel_off); free(c->lm_off); free(c->f_index); free(c->lm_ptr); free(c->lm_obs);
    free(c->col_size); free(c->col_pos); free(c->col_red); free(c->row_size); free(c->row_pos); free(c->row_cell);
    free(c->row_src); free(c->cell_col); free(c->cell_off); free(c->cell_src); free(c->values); free(c->bvec);
    free(c->obs_tmp); free(c->obs_ok);
}

/* cost of the residual blocks whose parameters are all constant (program.cc:305-390) */
static double ba_fixed_cost(ba_ctx* c) {
    double fc = 0.0;
    for (int o = 0; o < c->N; ++o) {
        if (c->obs_active[o]) continue;
        double cst, r[2];
        if (ba_eval_obs(c, o, &cst, r, NULL, NULL)) fc += cst;
    }
    return fc;
}

static void ba_pack(ba_ctx* c, double* x) {
    for (int k = 0; k < c->K; ++k) {
        if (c->pose_off[k] >= 0) memcpy(x + c->pose_off[k], c->pose_val + 6 * k, 6 * sizeof(double));
        if (c->vel_off[k] >= 0) memcpy(x + c->vel_off[k], c->vel_val + 3 * k, 3 * sizeof(double));
    }
    for (int l = 0; l < c->L; ++l)
        if (c->lm_off[l] >= 0) memcpy(x + c->lm_off[l], c->lm_val + 3 * l, 3 * sizeof(double));
    if (c->bg_off >= 0) memcpy(x + c->bg_off, c->bg_val, 3 * sizeof(double));
    if (c->ba_off >= 0) memcpy(x + c->ba_off, c->ba_val, 3 * sizeof(double));
}

/* one ceres::Solve on the current block values; updates them in place */
static void ba_ceres_solve(ba_ctx* c, const lm_options* base, lm_summary* sum) {
    lm_options opt = *base;
    opt.fixed_cost = ba_fixed_cost(c);
    if (c->n == 0) {
        memset(sum, 0, sizeof *sum);
        sum->termination = VIO_TERM_CONVERGENCE;
        sum->initial_cost = sum->final_cost = opt.fixed_cost;
        return;
    }
    double* x = (double*)malloc(sizeof(double) * c->n);
    ba_pack(c, x);
    lm_problem P = {c->n, c, ba_eval, ba_solve, ba_model_change};
    oracle_lm_minimize(&P, &opt, x, sum);
    ba_unpack(c, x);
    free(x);
}

static void write_pose(const pose_ctx* pc, const double* delta, vio_pose* out) {
    double dR[9], dt[3];
    se3_exp(delta, dR, dt);
    se3_mul(pc->R_init, pc->t_init, dR, dt, out->R, out->t);
}

static void trace_append(vio_ba_output* out, const lm_summary* sum, int* n) {
    for (int i = 0; i < sum->trace_n && i < sum->iterations; ++i) {
        if (out->trace && *n < out->trace_cap) out->trace[*n] = sum->trace[i];
        (*n)++;
    }
}

int oracle_ba_solve(const vio_ba_problem* p, vio_ba_output* out) {
    if (!p || !out || p->num_kf <= 0 || p->num_lm < 0 || p->num_obs < 0) return VIO_EINVAL;
    if (p->variant == VIO_BA_VI && (!p->preint || !p->preint_valid || !p->vel)) return VIO_EINVAL;
    ba_ctx c;
    ba_ctx_build(&c, p);
    lm_options opt;
    oracle_lm_default_options(&opt);
    opt.max_iterations = p->max_iterations;
    opt.fixed_iterations = p->fixed_iterations;
    lm_summary sum;
    vio_ba_summary S;
    memset(&S, 0, sizeof S);
    int N = c.N, L = c.L, K = c.K;
    double* chi2 = (double*)malloc(sizeof(double) * (N > 0 ? N : 1));
    uint8_t* outl = (uint8_t*)calloc(N > 0 ? N : 1, 1);
    const uint8_t* marg = c.is_pnp ? p->lm_const : p->lm_marg;

    int trace_n = 0;
    if (c.is_pnp) {
        int rounds = p->num_rounds > 0 ? p->num_rounds : 4;
        for (int round = 0; round < rounds; ++round) {
            memset(c.pose_val, 0, sizeof(double) * 6 * K);
            ba_ceres_solve(&c, &opt, &sum);
            trace_append(out, &sum, &trace_n);
            if (round == 0) S.initial_cost = sum.initial_cost;
            S.iterations += sum.iterations;
            S.num_successful_steps += sum.successful;
            S.num_unsuccessful_steps += sum.unsuccessful;
            int nin = 0, nout = 0;
            double inl_sum = 0;
            for (int o = 0; o < N; ++o) {
                int k = p->obs_kf[o], l = p->obs_lm[o];
                double ch = factor_chi2(&c.pc[k], c.pose_val + 6 * k, c.lm_val + 3 * l, (double)p->obs_uv[2 * o],
                                        (double)p->obs_uv[2 * o + 1], p->cols, p->rows, c.info, c.obs_outlier[o], 1);
                int m = marg ? marg[l] : 0;
                int is_out = !m && (ch > p->chi2_threshold);
                chi2[o] = ch;
                c.obs_outlier[o] = (uint8_t)is_out;
                if (is_out) nout++;
                else { nin++; inl_sum += ch; }
            }
            S.num_inliers = nin;
            S.num_outliers = nout;
            S.termination = sum.termination;
            S.success = sum.termination != VIO_TERM_FAILURE;
            S.final_cost = sum.final_cost;
            if (nin > 0) S.final_cost = inl_sum / nin;
        }
        memcpy(outl, c.obs_outlier, N);
        if (S.num_inliers < 10) S.success = 0;
        S.fixed_cost = 0;
    } else {
        ba_ceres_solve(&c, &opt, &sum);
        trace_append(out, &sum, &trace_n);
        S.initial_cost = sum.initial_cost;
        S.final_cost = sum.final_cost;
        S.iterations = sum.iterations;
        S.num_successful_steps = sum.successful;
        S.num_unsuccessful_steps = sum.unsuccessful;
        S.termination = sum.termination;
        S.success = sum.termination != VIO_TERM_FAILURE;
        S.fixed_cost = opt.fixed_cost; /* recomputed inside; same value */
        S.fixed_cost = ba_fixed_cost(&c);
        int* lin = (int*)calloc(L > 0 ? L : 1, sizeof(int));
        int* lout = (int*)calloc(L > 0 ? L : 1, sizeof(int));
        for (int o = 0; o < N; ++o) {
            int k = p->obs_kf[o], l = p->obs_lm[o];
            double ch = factor_chi2(&c.pc[k], c.pose_val + 6 * k, c.lm_val + 3 * l, (double)p->obs_uv[2 * o],
                                    (double)p->obs_uv[2 * o + 1], p->cols, p->rows, c.info, 0, 0);
            chi2[o] = ch;
            int is_out = ch > p->chi2_threshold;
            outl[o] = (uint8_t)is_out;
            if (is_out) { S.num_outliers++; lout[l]++; }
            else { S.num_inliers++; lin[l]++; }
        }
        for (int l = 0; l < L; ++l) {
            int m = marg ? marg[l] : 0;
            int bad = !m && lin[l] == 0 && lout[l] >= 2;
            if (out->lm_bad) out->lm_bad[l] = (uint8_t)bad;
            S.num_bad_lm += bad;
        }
        free(lin); free(lout);
    }
    if (out->T_wb)
        for (int k = 0; k < K; ++k) write_pose(&c.pc[k], c.pose_val + 6 * k, &out->T_wb[k]);
    if (out->lm_xyz) memcpy(out->lm_xyz, c.lm_val, sizeof(double) * 3 * L);
    if (out->obs_chi2) memcpy(out->obs_chi2, chi2, sizeof(double) * N);
    if (out->obs_outlier) memcpy(out->obs_outlier, outl, N);
    if (c.is_pnp && out->lm_bad) memset(out->lm_bad, 0, L);
    if (c.is_vi) {
        if (out->vel) memcpy(out->vel, c.vel_val, sizeof(double) * 3 * K);
        if (out->bg) memcpy(out->bg, c.bg_val, sizeof(double) * 3);
        if (out->ba) memcpy(out->ba, c.ba_val, sizeof(double) * 3);
    }
    if (out->summary) *out->summary = S;
    free(chi2); free(outl);
    ba_ctx_free(&c);
    return VIO_OK;
}

/* ========================================================================================= */
/* Test hooks for the restated Ceres known-answer tests                                       */
/* ========================================================================================= */
/* Powell's singular function (trust_region_minimizer_test.cc:262-294): dense 4x4 problem */
typedef struct { double J[16], r[4]; } powell_ctx;
static void powell_residuals(const double* x, double* r, double* J) {
    double x1 = x[0], x2 = x[1], x3 = x[2], x4 = x[3];
    r[0] = x1 + 10.0 * x2;
    r[1] = sqrt(5.0) * (x3 - x4);
    r[2] = (x2 - 2.0 * x3) * (x2 - 2.0 * x3);
    r[3] = sqrt(10.0) * (x1 - x4) * (x1 - x4);
    if (J) {
        memset(J, 0, 16 * sizeof(double));
        J[0] = 1.0; J[1] = 10.0;
        J[6] = sqrt(5.0); J[7] = -sqrt(5.0);
        J[9] = 2.0 * (x2 - 2.0 * x3); J[10] = -4.0 * (x2 - 2.0 * x3);
        J[12] = 2.0 * sqrt(10.0) * (x1 - x4); J[15] = -2.0 * sqrt(10.0) * (x1 - x4);
    }
}
static int powell_eval(void* u, const double* x, double* cost, int want, double* g, double* colsq) {
    powell_ctx* c = (powell_ctx*)u;
    double r[4], J[16];
    powell_residuals(x, r, J);
    *cost = 0.5 * (r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3]);
    if (want) {
        memcpy(c->J, J, sizeof J);
        memcpy(c->r, r, sizeof r);
        for (int j = 0; j < 4; ++j) {
            g[j] = 0; colsq[j] = 0;
            for (int i = 0; i < 4; ++i) { g[j] += J[4 * i + j] * r[i]; colsq[j] += J[4 * i + j] * J[4 * i + j]; }
        }
    }
    return 1;
}
static int powell_solve(void* u, const double* s, const double* D, double* y) {
    powell_ctx* c = (powell_ctx*)u;
    double A[16] = {0}, b[4] = {0};
    for (int a = 0; a < 4; ++a) {
        for (int i = 0; i < 4; ++i) b[a] += c->J[4 * i + a] * s[a] * c->r[i];
        for (int bb = 0; bb < 4; ++bb)
            for (int i = 0; i < 4; ++i) A[4 * a + bb] += c->J[4 * i + a] * s[a] * c->J[4 * i + bb] * s[bb];
        A[5 * a] += D[a] * D[a];
    }
    if (dense_llt(4, A) != 0) return 0;
    dense_llt_solve(4, A, b);
    memcpy(y, b, sizeof b);
    return 1;
}
static double powell_model(void* u, const double* s, const double* h) {
    powell_ctx* c = (powell_ctx*)u;
    double mc = 0;
    for (int i = 0; i < 4; ++i) {
        double m = 0;
        for (int j = 0; j < 4; ++j) m += c->J[4 * i + j] * s[j] * h[j];
        mc -= m * (c->r[i] + m / 2.0);
    }
    return mc;
}
/* IsTrustRegionSolveSuccessful<col1..col4> (trust_region_minimizer_test.cc:224-266) */
typedef struct { powell_ctx base; int mask[4]; int na; } powell_masked;
static void powell_full(const powell_masked* m, const double* xa, double* x4) {
    static const double zero = 0.0;
    (void)zero;
    int q = 0;
    for (int i = 0; i < 4; ++i) x4[i] = m->mask[i] ? xa[q++] : 0.0;
}
static int powellm_eval(void* u, const double* xa, double* cost, int want, double* g, double* colsq) {
    powell_masked* m = (powell_masked*)u;
    double x4[4], g4[4], c4[4];
    powell_full(m, xa, x4);
    powell_eval(&m->base, x4, cost, want, g4, c4);
    if (want) {
        int q = 0;
        for (int i = 0; i < 4; ++i)
            if (m->mask[i]) { g[q] = g4[i]; colsq[q] = c4[i]; q++; }
    }
    return 1;
}
/* DENSE_QR as in the Ceres test: Householder QR of the augmented [J~; D] (dense_qr_solver.cc) */
static int powellm_solve(void* u, const double* s, const double* D, double* y) {
    powell_masked* m = (powell_masked*)u;
    int na = m->na, cols[4], q = 0;
    for (int i = 0; i < 4; ++i)
        if (m->mask[i]) cols[q++] = i;
    int rows = 4 + na;
    double A[8][4] = {{0}}, b[8] = {0};
    for (int i = 0; i < 4; ++i) {
        for (int j = 0; j < na; ++j) A[i][j] = m->base.J[4 * i + cols[j]] * s[j];
        b[i] = m->base.r[i];
    }
    for (int j = 0; j < na; ++j) A[4 + j][j] = D[j];
    for (int j = 0; j < na; ++j) {
        double nrm = 0;
        for (int i = j; i < rows; ++i) nrm += A[i][j] * A[i][j];
        nrm = sqrt(nrm);
        if (nrm == 0.0) return 0;
        double alpha = A[j][j] > 0 ? -nrm : nrm;
        double v[8] = {0};
        for (int i = j; i < rows; ++i) v[i] = A[i][j];
        v[j] -= alpha;
        double vn = 0;
        for (int i = j; i < rows; ++i) vn += v[i] * v[i];
        if (vn == 0.0) continue;
        for (int c = j; c < na; ++c) {
            double d = 0;
            for (int i = j; i < rows; ++i) d += v[i] * A[i][c];
            d = 2.0 * d / vn;
            for (int i = j; i < rows; ++i) A[i][c] -= d * v[i];
        }
        double d = 0;
        for (int i = j; i < rows; ++i) d += v[i] * b[i];
        d = 2.0 * d / vn;
        for (int i = j; i < rows; ++i) b[i] -= d * v[i];
    }
    for (int j = na - 1; j >= 0; --j) {
        double t = b[j];
        for (int c = j + 1; c < na; ++c) t -= A[j][c] * y[c];
        y[j] = t / A[j][j];
    }
    return 1;
}
static double powellm_model(void* u, const double* s, const double* h) {
    powell_masked* m = (powell_masked*)u;
    int cols[4], q = 0;
    for (int i = 0; i < 4; ++i)
        if (m->mask[i]) cols[q++] = i;
    double mc = 0;
    for (int i = 0; i < 4; ++i) {
        double mm = 0;
        for (int j = 0; j < m->na; ++j) mm += m->base.J[4 * i + cols[j]] * s[j] * h[j];
        mc -= mm * (m->base.r[i] + mm / 2.0);
    }
    return mc;
}
/* x: 4 values in/out (inactive entries are forced to 0, the optimum) */
int oracle_powell(const int* mask, double* x, int* iterations, double* final_cost, int* termination) {
    powell_masked m;
    m.na = 0;
    for (int i = 0; i < 4; ++i) { m.mask[i] = mask[i] != 0; m.na += m.mask[i]; }
    double xa[4];
    int q = 0;
    for (int i = 0; i < 4; ++i)
        if (m.mask[i]) xa[q++] = x[i];
    lm_problem P = {m.na, &m, powellm_eval, powellm_solve, powellm_model};
    lm_options o;
    oracle_lm_default_options(&o);
    o.function_tolerance = 1e-26;
    o.gradient_tolerance = 1e-26;
    o.parameter_tolerance = 1e-26;
    o.initial_radius = 1e4;
    o.max_radius = 1e20;
    lm_summary s;
    oracle_lm_minimize(&P, &o, xa, &s);
    powell_full(&m, xa, x);
    *iterations = s.iterations;
    *final_cost = s.final_cost;
    *termination = s.termination;
    return 0;
}

/* DENSE_QR (dense_qr_solver.cc): Householder QR of the augmented [J~; diag(D)] (m + n rows),
   y = argmin |J~ y - r|^2 + |D y|^2.  Returns 0 on a zero column. */
static int dense_qr_lm_solve(int m, int n, const double* Js /* m x n */, const double* r, const double* D, double* y) {
    const int rows = m + n;
    double* A = (double*)calloc((size_t)rows * n, sizeof(double));
    double* b = (double*)calloc(rows, sizeof(double));
    double* v = (double*)malloc(sizeof(double) * rows);
    memcpy(A, Js, sizeof(double) * m * n);
    memcpy(b, r, sizeof(double) * m);
    for (int j = 0; j < n; ++j) A[(m + j) * n + j] = D ? D[j] : 0.0;
    int ok = 1;
    for (int j = 0; j < n && ok; ++j) {
        double nrm = 0;
        for (int i = j; i < rows; ++i) nrm += A[i * n + j] * A[i * n + j];
        nrm = sqrt(nrm);
        if (nrm == 0.0) { ok = 0; break; }
        const double alpha = A[j * n + j] > 0 ? -nrm : nrm;
        for (int i = 0; i < rows; ++i) v[i] = i >= j ? A[i * n + j] : 0.0;
        v[j] -= alpha;
        double vn = 0;
        for (int i = j; i < rows; ++i) vn += v[i] * v[i];
        if (vn == 0.0) continue;
        for (int c = j; c < n; ++c) {
            double d = 0;
            for (int i = j; i < rows; ++i) d += v[i] * A[i * n + c];
            d = 2.0 * d / vn;
            for (int i = j; i < rows; ++i) A[i * n + c] -= d * v[i];
        }
        double d = 0;
        for (int i = j; i < rows; ++i) d += v[i] * b[i];
        d = 2.0 * d / vn;
        for (int i = j; i < rows; ++i) b[i] -= d * v[i];
    }
    if (ok)
        for (int j = n - 1; j >= 0; --j) {
            double t = b[j];
            for (int c = j + 1; c < n; ++c) t -= A[j * n + c] * y[c];
            y[j] = t / A[j * n + j];
        }
    free(A); free(b); free(v);
    return ok;
}

/* JacobiScalingTest (trust_region_minimizer_test.cc:325-410): CurveCostFunction, one residual
   target - sum_i |y_i - y_{i-1}| over a closed polygon of nv 2-D vertices (y_{-1} = y_{nv-1}),
   solved by LM + DENSE_QR with the default Solver::Options (Jacobi scaling on). */
typedef struct { int nv; double target; double J[64]; double r; } curve_ctx;
static void curve_eval_rj(const curve_ctx* c, const double* y, double* r, double* J) {
    const int nv = c->nv;
    double res = c->target;
    for (int i = 0; i < nv; ++i) {
        const int prev = (nv + i - 1) % nv;
        double len = 0.0;
        for (int d = 0; d < 2; ++d) { const double diff = y[2 * prev + d] - y[2 * i + d]; len += diff * diff; }
        res -= sqrt(len);
    }
    *r = res;
    if (!J) return;
    for (int i = 0; i < nv; ++i) {
        const int prev = (nv + i - 1) % nv, next = (i + 1) % nv;
        double u[2], v[2], nu = 0, nvv = 0;
        for (int d = 0; d < 2; ++d) {
            u[d] = y[2 * i + d] - y[2 * prev + d]; nu += u[d] * u[d];
            v[d] = y[2 * next + d] - y[2 * i + d]; nvv += v[d] * v[d];
        }
        nu = sqrt(nu); nvv = sqrt(nvv);
        for (int d = 0; d < 2; ++d) {
            double j = 0.0;
            if (nu > DBL_MIN) j -= u[d] / nu;
            if (nvv > DBL_MIN) j += v[d] / nvv;
            J[2 * i + d] = j;
        }
    }
}
static int curve_eval(void* u, const double* x, double* cost, int want, double* g, double* colsq) {
    curve_ctx* c = (curve_ctx*)u;
    double r, J[64];
    curve_eval_rj(c, x, &r, want ? J : NULL);
    *cost = 0.5 * r * r;
    if (want) {
        c->r = r;
        memcpy(c->J, J, sizeof(double) * 2 * c->nv);
        for (int j = 0; j < 2 * c->nv; ++j) { g[j] = J[j] * r; colsq[j] = J[j] * J[j]; }
    }
    return 1;
}
static int curve_solve(void* u, const double* s, const double* D, double* y) {
    curve_ctx* c = (curve_ctx*)u;
    double Js[64];
    for (int j = 0; j < 2 * c->nv; ++j) Js[j] = c->J[j] * s[j];
    return dense_qr_lm_solve(1, 2 * c->nv, Js, &c->r, D, y);
}
static double curve_model(void* u, const double* s, const double* h) {
    curve_ctx* c = (curve_ctx*)u;
    double m = 0;
    for (int j = 0; j < 2 * c->nv; ++j) m += c->J[j] * s[j] * h[j];
    return -(m * (c->r + m / 2.0));
}
/* y: 2 nv values in/out */
int oracle_curve_kat(int nv, double target, double* y, double* final_cost, int* iterations, int* termination) {
    if (nv < 3 || nv > 32) return VIO_EINVAL;
    curve_ctx c;
    c.nv = nv;
    c.target = target;
    lm_problem P = {2 * nv, &c, curve_eval, curve_solve, curve_model};
    lm_options o;
    oracle_lm_default_options(&o);
    lm_summary sum;
    oracle_lm_minimize(&P, &o, y, &sum);
    *final_cost = sum.final_cost;
    *iterations = sum.iterations;
    *termination = sum.termination;
    return 0;
}

/* radius schedule hook: apply a sequence of accept(q>0)/reject(q<=0) events */
void oracle_lm_radius_schedule(double initial_radius, double max_radius, const double* q, int n, double* radii) {
    lm_radius s = {initial_radius, 2.0, max_radius};
    for (int i = 0; i < n; ++i) {
        if (q[i] > 0) oracle_lm_step_accepted(&s, q[i]);
        else oracle_lm_step_rejected(&s);
        radii[i] = s.radius;
    }
}

/* ========================================================================================= */
/* IMU initialisation: Optimizer::OptimizeIMUInit (src/optimization/Optimizer.cpp:972-1257)   */
/* over InertialGravityScaleFactor (src/optimization/Factors.cpp:981-1293) and BiasPriorFactor */
/* (src/optimization/Factors.h:366-396), LM + DENSE_QR with the default Solver::Options.       */
/* ========================================================================================= */

/* SO3d::Log (LieUtils.cpp:221-272) */
static void so3d_log(const double* R, double* w) {
    const double tr = R[0] + R[4] + R[8];
    const double c = fmax(-1.0, fmin(1.0, (tr - 1.0) * 0.5));
    const double th = acos(c);
    if (th < EPS_D) { /* Veed(R - I) */
        w[0] = R[7]; w[1] = R[2]; w[2] = R[3];
        return;
    }
    const double s = sin(th);
    if (fabs(s) < EPS_D) {
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

/* InertialGravityScaleFactor::log_SO3 (Factors.cpp:1235-1241): SVD re-orthonormalisation, the
   SO3d constructor's second one, SO3d::Log */
static void igs_log_so3(const double* R, double* w) {
    double R1[9], R2[9];
    oracle_nearest_rotation(R, R1);
    oracle_nearest_rotation(R1, R2);
    so3d_log(R2, w);
}

/* InertialGravityScaleFactor::right_jacobian_SO3 (Factors.cpp:1207-1220): I - skew/2 below 1e-6 */
static void igs_right_jac(const double* phi, double* J) {
    double P[9];
    hat3(phi, P);
    const double th = norm3(phi);
    if (th < 1e-6) {
        for (int i = 0; i < 9; ++i) J[i] = ((i % 4 == 0) ? 1.0 : 0.0) - 0.5 * P[i];
        return;
    }
    double P2[9];
    m3_mul(P, P, P2);
    const double c = cos(th), s = sin(th);
    for (int i = 0; i < 9; ++i) J[i] = ((i % 4 == 0) ? 1.0 : 0.0) - P[i] * (1.0 - c) / (th * th) + P2[i] * (th - s) / (th * th * th);
}

/* Eigen's 3x3 inverse (cofactors, det along column 0) */
static void inv3_eigen(const double* m, double* r) {
#define M3(i, j) m[3 * (i) + (j)]
#define COF(i, j) (M3(((i) + 1) % 3, ((j) + 1) % 3) * M3(((i) + 2) % 3, ((j) + 2) % 3) - \
                   M3(((i) + 1) % 3, ((j) + 2) % 3) * M3(((i) + 2) % 3, ((j) + 1) % 3))
    const double c0[3] = {COF(0, 0), COF(1, 0), COF(2, 0)};
    const double det = c0[0] * M3(0, 0) + c0[1] * M3(1, 0) + c0[2] * M3(2, 0);
    const double id = 1.0 / det;
    for (int j = 0; j < 3; ++j) r[j] = c0[j] * id;
    for (int i = 1; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[3 * i + j] = COF(j, i) * id;
#undef COF
#undef M3
}

/* gravity_dir_to_rotation (Factors.cpp:1243-1266) */
static void igs_gdir_rot(const double* gd, double* R) {
    const double w[3] = {gd[0], gd[1], 0.0};
    const double d2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    const double d = sqrt(d2);
    double W[9], W2[9];
    hat3(w, W);
    m3_mul(W, W, W2);
    for (int i = 0; i < 9; ++i) {
        const double I = (i % 4 == 0) ? 1.0 : 0.0;
        R[i] = d < 1e-5 ? I + W[i] + 0.5 * W2[i] : I + W[i] * sin(d) / d + W2[i] * (1.0 - cos(d)) / d2;
    }
}

typedef struct {
    double dR[9], dV[3], dP[3], JRg[9], JVg[9], JVa[9], JPg[9], JPa[9], bg0[3], ba0[3], dt;
    int i; /* links frame i -> i + 1 */
} igs_factor;

typedef struct {
    int F, stage, nf, n, m;
    igs_factor* fac;
    double gm, huber, prior_w;
    /* parameter values */
    double* vel; /* 3F */
    double bg[3], ba[3], gdir[2], scale;
    /* stage-2 layout: offset of vel_k / bg / ba in x (first appearance), -1 if absent */
    int* vel_off;
    int bg_off, ba_off;
    double* J;   /* m x n (corrected), row-major */
    double* r;   /* m */
    double* Js;  /* m x n scratch */
} igs_ctx;

/* InertialGravityScaleFactor::Evaluate (Factors.cpp:1015-1180) at identity poses: residual (9) and
   the Jacobian blocks of vel_i, bg, ba, vel_j (3 cols each), gravity_dir (2), scale (1) */
static void igs_eval_factor(const igs_ctx* c, const igs_factor* f, double* r, double* Jvi, double* Jbg, double* Jba,
                            double* Jvj, double* Jgd, double* Jsc) {
    const double* vi = c->vel + 3 * f->i;
    const double* vj = c->vel + 3 * (f->i + 1);
    const double s = c->scale, dt = f->dt;
    double Rwg[9], g[3];
    igs_gdir_rot(c->gdir, Rwg);
    for (int k = 0; k < 3; ++k) g[k] = Rwg[3 * k + 2] * -c->gm;
    double dR[9], dV[3], dP[3], dbg[3], dba[3];
    memcpy(dR, f->dR, sizeof dR); memcpy(dV, f->dV, sizeof dV); memcpy(dP, f->dP, sizeof dP);
    for (int k = 0; k < 3; ++k) { dbg[k] = c->bg[k] - f->bg0[k]; dba[k] = c->ba[k] - f->ba0[k]; }
    if (norm3(dbg) > 1e-6 || norm3(dba) > 1e-6) {
        double w[3], E[9], M[9];
        m3_vec(f->JRg, dbg, w);
        so3_exp(w, E);
        m3_mul(dR, E, M);
        memcpy(dR, M, sizeof M);
        double a[3], b[3];
        m3_vec(f->JVg, dbg, a); m3_vec(f->JVa, dba, b);
        for (int k = 0; k < 3; ++k) dV[k] = dV[k] + a[k] + b[k];
        m3_vec(f->JPg, dbg, a); m3_vec(f->JPa, dba, b);
        for (int k = 0; k < 3; ++k) dP[k] = dP[k] + a[k] + b[k];
    }
    double eR[9];
    m3_tr(dR, eR); /* delta_R^T * R_bwi * R_wbj with identity poses */
    double er[3];
    igs_log_so3(eR, er);
    for (int k = 0; k < 3; ++k) {
        r[k] = er[k];
        r[3 + k] = (s * (vj[k] - vi[k]) - g[k] * dt) - dV[k];
        r[6 + k] = (s * (0.0 - vi[k] * dt) - 0.5 * g[k] * dt * dt) - dP[k];
    }
    if (!Jvi) return;
    /* 9x3 row-major blocks */
    memset(Jvi, 0, 27 * sizeof(double)); memset(Jbg, 0, 27 * sizeof(double)); memset(Jba, 0, 27 * sizeof(double));
    memset(Jvj, 0, 27 * sizeof(double)); memset(Jgd, 0, 18 * sizeof(double)); memset(Jsc, 0, 9 * sizeof(double));
    for (int k = 0; k < 3; ++k) {
        Jvi[3 * (3 + k) + k] = -s;
        Jvi[3 * (6 + k) + k] = -s * dt;
        Jvj[3 * (3 + k) + k] = s;
    }
    double Jr[9], Jri[9], Jb[9], t1[9], t2[9], t3[9], w[3], eRt[9];
    igs_right_jac(er, Jr);
    inv3_eigen(Jr, Jri);
    m3_vec(f->JRg, dbg, w);
    igs_right_jac(w, Jb);
    m3_tr(eR, eRt);
    for (int i = 0; i < 9; ++i) t1[i] = -Jri[i];
    m3_mul(t1, eRt, t2);
    m3_mul(t2, Jb, t3);
    m3_mul(t3, f->JRg, t1);
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
            Jbg[3 * a + b] = t1[3 * a + b];
            Jbg[3 * (3 + a) + b] = -f->JVg[3 * a + b];
            Jbg[3 * (6 + a) + b] = -f->JPg[3 * a + b];
            Jba[3 * (3 + a) + b] = -f->JVa[3 * a + b];
            Jba[3 * (6 + a) + b] = -f->JPa[3 * a + b];
        }
    /* dg/dtheta = R_wg * [[0, -gm], [gm, 0], [0, 0]] */
    for (int k = 0; k < 3; ++k) {
        const double d0 = Rwg[3 * k + 1] * c->gm, d1 = Rwg[3 * k] * -c->gm;
        Jgd[2 * (3 + k)] = -d0 * dt;
        Jgd[2 * (3 + k) + 1] = -d1 * dt;
        Jgd[2 * (6 + k)] = -0.5 * d0 * dt * dt;
        Jgd[2 * (6 + k) + 1] = -0.5 * d1 * dt * dt;
        Jsc[3 + k] = vj[k] - vi[k];
        Jsc[6 + k] = 0.0 - vi[k] * dt;
    }
}

static void igs_unpack(igs_ctx* c, const double* x) {
    if (c->stage == 1) {
        c->gdir[0] = x[0]; c->gdir[1] = x[1]; c->scale = x[2];
        return;
    }
    for (int k = 0; k < c->F; ++k)
        if (c->vel_off[k] >= 0) memcpy(c->vel + 3 * k, x + c->vel_off[k], 3 * sizeof(double));
    memcpy(c->bg, x + c->bg_off, 3 * sizeof(double));
    memcpy(c->ba, x + c->ba_off, 3 * sizeof(double));
}

static int igs_eval(void* user, const double* x, double* cost, int want_jac, double* g, double* colsq) {
    igs_ctx* c = (igs_ctx*)user;
    const int n = c->n;
    igs_unpack(c, x);
    double total = 0.0;
    if (want_jac) memset(c->J, 0, sizeof(double) * (size_t)c->m * n);
    for (int q = 0; q < c->nf; ++q) {
        double r[9], B[6][27];
        igs_eval_factor(c, &c->fac[q], r, want_jac ? B[0] : NULL, B[1], B[2], B[3], B[4], B[5]);
        double sq = 0;
        for (int i = 0; i < 9; ++i) sq += r[i] * r[i];
        double rho[3];
        oracle_huber(c->huber, sq, rho);
        total += 0.5 * rho[0];
        double rs, asq, sr1;
        oracle_corrector(sq, rho, &rs, &asq, &sr1);
        if (want_jac) {
            /* scatter the free columns: stage 1 gdir(2), scale; stage 2 vel_i, bg, ba, vel_j */
            double* row = c->J + (size_t)9 * q * n;
            if (c->stage == 1) {
                for (int i = 0; i < 9; ++i) { row[i * n] = B[4][2 * i]; row[i * n + 1] = B[4][2 * i + 1]; row[i * n + 2] = B[5][i]; }
            } else {
                const int offs[4] = {c->vel_off[c->fac[q].i], c->bg_off, c->ba_off, c->vel_off[c->fac[q].i + 1]};
                for (int b = 0; b < 4; ++b)
                    for (int i = 0; i < 9; ++i)
                        for (int j = 0; j < 3; ++j) row[i * n + offs[b] + j] = B[b][3 * i + j];
            }
            /* Corrector::CorrectJacobian over the block's columns (residual_block.cc:178-189) */
            for (int col = 0; col < n; ++col) {
                if (asq == 0.0) {
                    for (int i = 0; i < 9; ++i) row[i * n + col] *= sr1;
                } else {
                    double rtj = 0;
                    for (int i = 0; i < 9; ++i) rtj += row[i * n + col] * r[i];
                    for (int i = 0; i < 9; ++i) row[i * n + col] = sr1 * (row[i * n + col] - asq * r[i] * rtj);
                }
            }
            for (int i = 0; i < 9; ++i) c->r[9 * q + i] = r[i] * rs;
        }
    }
    if (c->stage == 2) { /* BiasPriorFactor x2 (gyro, accel), no loss */
        for (int b = 0; b < 2; ++b) {
            const double* v = b ? c->ba : c->bg;
            const int off = b ? c->ba_off : c->bg_off;
            double sq = 0, r[3];
            for (int k = 0; k < 3; ++k) { r[k] = c->prior_w * (v[k] - 0.0); sq += r[k] * r[k]; }
            total += 0.5 * sq;
            if (want_jac) {
                const int row0 = 9 * c->nf + 3 * b;
                for (int k = 0; k < 3; ++k) {
                    c->J[(size_t)(row0 + k) * n + off + k] = c->prior_w;
                    c->r[row0 + k] = r[k];
                }
            }
        }
    }
    if (want_jac) {
        memset(g, 0, sizeof(double) * n);
        memset(colsq, 0, sizeof(double) * n);
        for (int i = 0; i < c->m; ++i)
            for (int j = 0; j < n; ++j) {
                g[j] += c->J[(size_t)i * n + j] * c->r[i];
                colsq[j] += c->J[(size_t)i * n + j] * c->J[(size_t)i * n + j];
            }
    }
    *cost = total;
    return 1;
}

static int igs_solve(void* user, const double* s, const double* D, double* y) {
    igs_ctx* c = (igs_ctx*)user;
    for (int i = 0; i < c->m; ++i)
        for (int j = 0; j < c->n; ++j) c->Js[(size_t)i * c->n + j] = c->J[(size_t)i * c->n + j] * s[j];
    return dense_qr_lm_solve(c->m, c->n, c->Js, c->r, D, y);
}

static double igs_model(void* user, const double* s, const double* h) {
    igs_ctx* c = (igs_ctx*)user;
    double mc = 0;
    for (int i = 0; i < c->m; ++i) {
        double jh = 0;
        for (int j = 0; j < c->n; ++j) jh += c->J[(size_t)i * c->n + j] * (s[j] * h[j]);
        mc -= jh * (c->r[i] + jh / 2.0);
    }
    return mc;
}

int oracle_imu_init(const vio_imu_init_problem* p, vio_imu_init_result* out) {
    if (!p || !out) return VIO_EINVAL;
    double* vel_out = out->velocities;
    memset(out, 0, sizeof *out);
    out->velocities = vel_out;
    out->scale = 1.0;
    out->gravity[2] = (double)-9.81f;
    out->Rwg[0] = out->Rwg[4] = out->Rwg[8] = 1.0;
    const int F = p->num_frames;
    if (F < 3) { out->status = VIO_IMU_INIT_FEW_FRAMES; return VIO_OK; }
    if (!p->preint || !p->preint_valid || !p->T_wb) return VIO_EINVAL;
    for (int i = 1; i < F; ++i)
        if (!p->preint_valid[i]) { out->status = VIO_IMU_INIT_NO_PREINT; return VIO_OK; }
    igs_ctx c;
    memset(&c, 0, sizeof c);
    c.F = F;
    c.gm = p->gravity_magnitude;
    c.huber = p->huber_delta;
    c.prior_w = p->bias_prior_weight;
    c.scale = 1.0;
    c.vel = (double*)calloc(3 * (size_t)F, sizeof(double));
    c.vel_off = (int*)malloc(sizeof(int) * F);
    c.fac = (igs_factor*)calloc(F, sizeof(igs_factor));
    /* velocity initialisation from the preintegration: R_wb_prev * delta_V (:1025-1036) */
    for (int i = 1; i < F; ++i) {
        const vio_preint* q = &p->preint[i];
        if (q->dt_total > 0.001) {
            double dv[3] = {q->delta_V[0], q->delta_V[1], q->delta_V[2]};
            m3_vec(p->T_wb[i - 1].R, dv, c.vel + 3 * i);
        }
    }
    /* factors i -> i+1 with 0.001 <= dt <= 2.0 (:1058-1066) */
    for (int i = 0; i < F - 1; ++i) {
        const vio_preint* q = &p->preint[i + 1];
        if (q->dt_total < 0.001 || q->dt_total > 2.0) continue;
        igs_factor* f = &c.fac[c.nf++];
        f->i = i;
        f->dt = q->dt_total;
        for (int k = 0; k < 9; ++k) {
            f->dR[k] = q->delta_R[k];
            f->JRg[k] = q->J_Rg[k]; f->JVg[k] = q->J_Vg[k]; f->JVa[k] = q->J_Va[k];
            f->JPg[k] = q->J_Pg[k]; f->JPa[k] = q->J_Pa[k];
        }
        for (int k = 0; k < 3; ++k) {
            f->dV[k] = q->delta_V[k]; f->dP[k] = q->delta_P[k];
            f->bg0[k] = q->gyro_bias[k]; f->ba0[k] = q->accel_bias[k];
        }
    }
    if (c.nf == 0) {
        out->status = VIO_IMU_INIT_NO_FACTORS;
        free(c.vel); free(c.vel_off); free(c.fac);
        return VIO_OK;
    }
    lm_options opt;
    oracle_lm_default_options(&opt);
    opt.max_iterations = p->max_iterations;
    lm_summary* sum = (lm_summary*)malloc(sizeof(lm_summary));
    /* stage 1: gravity_dir + scale */
    {
        c.stage = 1;
        c.n = 3;
        c.m = 9 * c.nf;
        c.J = (double*)calloc((size_t)c.m * c.n, sizeof(double));
        c.Js = (double*)calloc((size_t)c.m * c.n, sizeof(double));
        c.r = (double*)calloc(c.m, sizeof(double));
        double x[3] = {c.gdir[0], c.gdir[1], c.scale};
        lm_problem P = {3, &c, igs_eval, igs_solve, igs_model};
        oracle_lm_minimize(&P, &opt, x, sum);
        igs_unpack(&c, x);
        out->initial_cost = sum->initial_cost;
        out->iterations[0] = sum->iterations;
        out->termination[0] = sum->termination;
        free(c.J); free(c.Js); free(c.r);
    }
    /* stage 2: velocities + biases (+ the two bias priors), in order of first appearance */
    {
        c.stage = 2;
        int off = 0;
        for (int k = 0; k < F; ++k) c.vel_off[k] = -1;
        c.bg_off = c.ba_off = -1;
        for (int q = 0; q < c.nf; ++q) {
            const int i = c.fac[q].i;
            if (c.vel_off[i] < 0) { c.vel_off[i] = off; off += 3; }
            if (c.bg_off < 0) { c.bg_off = off; off += 3; }
            if (c.ba_off < 0) { c.ba_off = off; off += 3; }
            if (c.vel_off[i + 1] < 0) { c.vel_off[i + 1] = off; off += 3; }
        }
        c.n = off;
        c.m = 9 * c.nf + 6;
        c.J = (double*)calloc((size_t)c.m * c.n, sizeof(double));
        c.Js = (double*)calloc((size_t)c.m * c.n, sizeof(double));
        c.r = (double*)calloc(c.m, sizeof(double));
        double* x = (double*)calloc(c.n, sizeof(double));
        for (int k = 0; k < F; ++k)
            if (c.vel_off[k] >= 0) memcpy(x + c.vel_off[k], c.vel + 3 * k, 3 * sizeof(double));
        memcpy(x + c.bg_off, c.bg, 3 * sizeof(double));
        memcpy(x + c.ba_off, c.ba, 3 * sizeof(double));
        lm_problem P = {c.n, &c, igs_eval, igs_solve, igs_model};
        oracle_lm_minimize(&P, &opt, x, sum);
        igs_unpack(&c, x);
        out->final_cost = sum->final_cost;
        out->iterations[1] = sum->iterations;
        out->termination[1] = sum->termination;
        free(x); free(c.J); free(c.Js); free(c.r);
    }
    /* results (:1212-1238): R_wg = AngleAxisd(|w|, w/|w|) for w = (theta_x, theta_y, 0) */
    const double om[3] = {c.gdir[0], c.gdir[1], 0.0};
    const double ang = sqrt(om[0] * om[0] + om[1] * om[1] + om[2] * om[2]);
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (!(ang < 1e-6)) {
        const double ax[3] = {om[0] / ang, om[1] / ang, om[2] / ang};
        const double sn = sin(ang), cs = cos(ang);
        const double sa[3] = {sn * ax[0], sn * ax[1], sn * ax[2]};
        const double ca[3] = {(1.0 - cs) * ax[0], (1.0 - cs) * ax[1], (1.0 - cs) * ax[2]};
        double t = ca[0] * ax[1];
        R[1] = t - sa[2]; R[3] = t + sa[2];
        t = ca[0] * ax[2];
        R[2] = t + sa[1]; R[6] = t - sa[1];
        t = ca[1] * ax[2];
        R[5] = t - sa[0]; R[7] = t + sa[0];
        R[0] = ca[0] * ax[0] + cs; R[4] = ca[1] * ax[1] + cs; R[8] = ca[2] * ax[2] + cs;
    }
    memcpy(out->Rwg, R, sizeof R);
    for (int k = 0; k < 3; ++k) out->gravity[k] = R[3 * k + 2] * -9.81;
    out->gravity_dir[0] = c.gdir[0];
    out->gravity_dir[1] = c.gdir[1];
    out->scale = c.scale;
    memcpy(out->gyro_bias, c.bg, sizeof c.bg);
    memcpy(out->accel_bias, c.ba, sizeof c.ba);
    if (vel_out) memcpy(vel_out, c.vel, sizeof(double) * 3 * F);
    out->success = 1;
    out->status = VIO_IMU_INIT_OK;
    free(sum); free(c.vel); free(c.vel_off); free(c.fac);
    return VIO_OK;
}

/* ========================================================================================= */
/* Lie maths test entry points (tests/test_lie_kat.py: Ceres rotation_test.cc known answers)   */
/* ========================================================================================= */
/* SO3d::Exp incl. the SO3d constructor's projection (LieUtils.cpp:203-219, 275-288) */
void oracle_so3_exp(const double* w, double* R) { so3_exp(w, R); }
/* SE3d::exp (LieUtils.cpp:305-333) */
void oracle_se3_exp(const double* xi, double* R, double* t) { se3_exp(xi, R, t); }
/* SO3d::Log (LieUtils.cpp:221-273) */
void oracle_so3d_log(const double* R, double* w) { so3d_log(R, w); }
/* InertialFactorFixedGravity::log_SO3 (Factors.cpp:1507-1519) */
void oracle_imu_log_so3(const double* R, double* w) { imu_log_so3(R, w); }
