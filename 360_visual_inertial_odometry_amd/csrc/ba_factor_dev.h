// ba_factor_dev.h — device maths of the ERP reprojection factor shared by the windowed solver
// (ba_kernel.hip) and the global-BA kernels (ba_global.hip).
#pragma once
#include <float.h>
#include <hip/hip_runtime.h>

#include "lie_dev.h"

namespace vio360 {

// pose cache at parameter xi: T_wb = SE3(T_init) * exp(xi) (Factors.cpp:351-364).
// pinit: projected R_init(9) t_init(3) R_cb(9) t_cb(3); pc: Rwb(9) twb(3) Rbw(9) tbw(3) Rcw(9) tcw(3)
__device__ __forceinline__ void pose_cache_one(const double* pinit, const double* xp, double* pc) {
    double dR[9], dt[3], xi[6];
    for (int i = 0; i < 6; ++i) xi[i] = xp[i];
    se3_exp(xi, dR, dt);
    const double* Ri = pinit;
    const double* ti = pinit + 9;
    const double* Rc = pinit + 12;
    const double* tc = pinit + 21;
    double Rwb[9], twb[3], Rbw[9], tbw[3], Rcw[9], tcw[3];
    m3mul(Ri, dR, Rwb);
    m3vec(Ri, dt, twb);
    for (int i = 0; i < 3; ++i) twb[i] += ti[i];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) Rbw[3 * i + j] = Rwb[3 * j + i];
    m3vec(Rbw, twb, tbw);
    for (int i = 0; i < 3; ++i) tbw[i] = -tbw[i];
    m3mul(Rc, Rbw, Rcw);
    m3vec(Rc, tbw, tcw);
    for (int i = 0; i < 3; ++i) tcw[i] += tc[i];
    for (int i = 0; i < 9; ++i) { pc[i] = Rwb[i]; pc[12 + i] = Rbw[i]; pc[24 + i] = Rcw[i]; }
    for (int i = 0; i < 3; ++i) { pc[9 + i] = twb[i]; pc[21 + i] = tbw[i]; pc[33 + i] = tcw[i]; }
}

// ------------------------------------------------------------------------------------------
// HuberLoss(delta) (loss_function.cc:48-62) -> cost, residual scale, Jacobian scale.
// rho'' <= 0 everywhere for Huber, so the Corrector reduces to sqrt(rho') scaling (corrector.cc:82-86).
__device__ __forceinline__ void huber(double delta, double sq, double& cost, double& scale) {
    double b = delta * delta;
    if (sq > b) {
        double r = sqrt(sq);
        cost = 0.5 * (2.0 * delta * r - b);
        scale = sqrt(fmax(DBL_MIN, delta / r));
    } else {
        cost = 0.5 * sq;
        scale = 1.0;
    }
}

// BAFactor::Evaluate / PnPFactor::Evaluate (Factors.cpp:33-210, 327-542) given the pose cache.
// returns 0 = ok, 1 = evaluation failure (PnP with |Pc| < 1e-10)
__device__ __forceinline__ int factor_eval(const double* pc, const double* Rcb_raw, const double* Pw, double uo,
                                           double vo, double cols, double rows, const double* Lw, bool outlier,
                                           bool is_pnp, bool want_jac, double* r, double* Jp, double* Jl,
                                           bool& jzero) {
    jzero = true;
    if (outlier) {
        r[0] = 640.0; r[1] = 480.0;
        return 0;
    }
    const double* Rbw = pc + 12;
    const double* tbw = pc + 21;
    const double* Rcw = pc + 24;
    const double* tcw = pc + 33;
    double Pc[3];
    m3vec(Rcw, Pw, Pc);
    Pc[0] += tcw[0]; Pc[1] += tcw[1]; Pc[2] += tcw[2];
    double x = Pc[0], y = Pc[1], z = Pc[2];
    double L = nrm3(Pc);
    if (L < 1e-10) {
        if (is_pnp) return 1;
        r[0] = 640.0; r[1] = 360.0;
        return 0;
    }
    // divisions by L, 2 pi, pi and the Jacobian denominators become products with reciprocals (2
    // divisions per evaluation instead of 8; each value moves by at most an ulp or two)
    constexpr double inv2pi = 1.0 / (2.0 * M_PI), invpi = 1.0 / M_PI;
    const double iL = 1.0 / L;
    double theta = atan2(x, z);
    double phi = -asin(y * iL);
    double u = cols * (0.5 + theta * inv2pi);
    double v = rows * (0.5 - phi * invpi);
    double du = uo - u, dv = vo - v;
    if (du > cols / 2.0) du -= cols;
    else if (du < -cols / 2.0) du += cols;
    if (fabs(du) > 100.0 || fabs(dv) > 100.0) {
        r[0] = 100.0; r[1] = 100.0;
        return 0;
    }
    r[0] = Lw[0] * du;
    r[1] = Lw[2] * du + Lw[3] * dv;
    if (!want_jac) return 0;
    double xz2 = x * x + z * z, L2 = L * L;
    if (xz2 < 1e-10 || L2 < 1e-10) return 0;
    jzero = false;
    double xzn = sqrt(xz2);
    const double ixzn = 1.0 / xzn, ixz2 = ixzn * ixzn, iL2 = iL * iL, iL2xzn = iL2 * ixzn;
    const double cu = cols * inv2pi, cv = rows * invpi;
    double Jc[6];
    Jc[0] = -cu * z * ixz2;
    Jc[1] = 0.0;
    Jc[2] = cu * x * ixz2;
    Jc[3] = cv * (x * y) * iL2xzn;
    Jc[4] = -cv * xzn * iL2;
    Jc[5] = cv * (y * z) * iL2xzn;
    double Jw[6];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        Jw[j] = Lw[0] * Jc[j];
        Jw[3 + j] = Lw[2] * Jc[j] + Lw[3] * Jc[3 + j];
    }
    // pose: [ -R_cb_raw | R_cb_raw [Pb]x ]   (Factors.cpp:500-522)
    double Pb[3];
    m3vec(Rbw, Pw, Pb);
    Pb[0] += tbw[0]; Pb[1] += tbw[1]; Pb[2] += tbw[2];
    double A[6];  // Jw * R_cb_raw (2x3)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            A[3 * i + j] = Jw[3 * i] * Rcb_raw[j] + Jw[3 * i + 1] * Rcb_raw[3 + j] + Jw[3 * i + 2] * Rcb_raw[6 + j];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const double* a = A + 3 * i;
        Jp[6 * i + 0] = -a[0];
        Jp[6 * i + 1] = -a[1];
        Jp[6 * i + 2] = -a[2];
        // a * hat(Pb): [a1*Pb2 - a2*Pb1... ] row vector times skew
        Jp[6 * i + 3] = a[1] * Pb[2] - a[2] * Pb[1];
        Jp[6 * i + 4] = a[2] * Pb[0] - a[0] * Pb[2];
        Jp[6 * i + 5] = a[0] * Pb[1] - a[1] * Pb[0];
        // point: Jw * R_cb_raw * R_bw   (Factors.cpp:525-534)
#pragma unroll
        for (int j = 0; j < 3; ++j) Jl[3 * i + j] = a[0] * Rbw[j] + a[1] * Rbw[3 + j] + a[2] * Rbw[6 + j];
    }
    return 0;
}

// The Jacobian tail of factor_eval_ap at camera-frame point (x, y, z), |P| = L, 1 / L = iL: A = Jw R_cb_raw
// (2x3, weighted) and Pb = R_bw Pw + t_bw.  Returns false (A, Pb untouched) where the Jacobian is zero.
__device__ __forceinline__ bool factor_ap_tail(double x, double y, double z, double L, double iL, const double* Rbw,
                                               const double* tbw, const double* Pw, const double* Rcb_raw, double cols,
                                               double rows, const double* Lw, double* A, double* Pb) {
    constexpr double inv2pi = 1.0 / (2.0 * M_PI), invpi = 1.0 / M_PI;
    double xz2 = x * x + z * z, L2 = L * L;
    if (xz2 < 1e-10 || L2 < 1e-10) return false;
    double xzn = sqrt(xz2);
    const double ixzn = 1.0 / xzn, ixz2 = ixzn * ixzn, iL2 = iL * iL, iL2xzn = iL2 * ixzn;
    const double cu = cols * inv2pi, cv = rows * invpi;
    double Jc[6];
    Jc[0] = -cu * z * ixz2;
    Jc[1] = 0.0;
    Jc[2] = cu * x * ixz2;
    Jc[3] = cv * (x * y) * iL2xzn;
    Jc[4] = -cv * xzn * iL2;
    Jc[5] = cv * (y * z) * iL2xzn;
    double Jw[6];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        Jw[j] = Lw[0] * Jc[j];
        Jw[3 + j] = Lw[2] * Jc[j] + Lw[3] * Jc[3 + j];
    }
    m3vec(Rbw, Pw, Pb);
    Pb[0] += tbw[0]; Pb[1] += tbw[1]; Pb[2] += tbw[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            A[3 * i + j] = Jw[3 * i] * Rcb_raw[j] + Jw[3 * i + 1] * Rcb_raw[3 + j] + Jw[3 * i + 2] * Rcb_raw[6 + j];
    return true;
}

// BAFactor::Evaluate as factor_eval, returning the Jacobian in compressed form: A = Jw R_cb_raw (2x3,
// weighted) and Pb (point in the body frame); J_pose / J_point follow as in jac_from_ap.
__device__ __forceinline__ int factor_eval_ap(const double* pc, const double* Rcb_raw, const double* Pw, double uo,
                                              double vo, double cols, double rows, const double* Lw, bool outlier,
                                              bool is_pnp, double* r, double* A, double* Pb, bool& jzero) {
    jzero = true;
    if (outlier) {
        r[0] = 640.0; r[1] = 480.0;
        return 0;
    }
    const double* Rbw = pc + 12;
    const double* tbw = pc + 21;
    const double* Rcw = pc + 24;
    const double* tcw = pc + 33;
    double Pc[3];
    m3vec(Rcw, Pw, Pc);
    Pc[0] += tcw[0]; Pc[1] += tcw[1]; Pc[2] += tcw[2];
    double x = Pc[0], y = Pc[1], z = Pc[2];
    double L = nrm3(Pc);
    if (L < 1e-10) {
        if (is_pnp) return 1;
        r[0] = 640.0; r[1] = 360.0;
        return 0;
    }
    // divisions by L, 2 pi, pi and the Jacobian denominators become products with reciprocals (2
    // divisions per evaluation instead of 8; each value moves by at most an ulp or two)
    constexpr double inv2pi = 1.0 / (2.0 * M_PI), invpi = 1.0 / M_PI;
    const double iL = 1.0 / L;
    double theta = atan2(x, z);
    double phi = -asin(y * iL);
    double u = cols * (0.5 + theta * inv2pi);
    double v = rows * (0.5 - phi * invpi);
    double du = uo - u, dv = vo - v;
    if (du > cols / 2.0) du -= cols;
    else if (du < -cols / 2.0) du += cols;
    if (fabs(du) > 100.0 || fabs(dv) > 100.0) {
        r[0] = 100.0; r[1] = 100.0;
        return 0;
    }
    r[0] = Lw[0] * du;
    r[1] = Lw[2] * du + Lw[3] * dv;
    jzero = !factor_ap_tail(x, y, z, L, iL, Rbw, tbw, Pw, Rcb_raw, cols, rows, Lw, A, Pb);
    return 0;
}

// factor_eval_ap in two parts: the residual (returns 1 on a PnP evaluation failure); `tail` says whether the
// Jacobian tail applies (factor_ap_tail at the camera-frame point P, |P| = L, 1 / L = iL), which the caller
// runs when it needs A / Pb -- after its loss, so that A / Pb are not live across it (the same operations
// as factor_eval_ap, hence the same values)
__device__ __forceinline__ int factor_eval_res(const double* pc, const double* Pw, double uo, double vo, double cols,
                                               double rows, const double* Lw, bool outlier, bool is_pnp, double* r,
                                               double* P, double& L, double& iL, bool& tail) {
    tail = false;
    if (outlier) {
        r[0] = 640.0; r[1] = 480.0;
        return 0;
    }
    const double* Rcw = pc + 24;
    const double* tcw = pc + 33;
    m3vec(Rcw, Pw, P);
    P[0] += tcw[0]; P[1] += tcw[1]; P[2] += tcw[2];
    const double x = P[0], y = P[1], z = P[2];
    L = nrm3(P);
    if (L < 1e-10) {
        if (is_pnp) return 1;
        r[0] = 640.0; r[1] = 360.0;
        return 0;
    }
    constexpr double inv2pi = 1.0 / (2.0 * M_PI), invpi = 1.0 / M_PI;
    iL = 1.0 / L;
    double theta = atan2(x, z);
    double phi = -asin(y * iL);
    double u = cols * (0.5 + theta * inv2pi);
    double v = rows * (0.5 - phi * invpi);
    double du = uo - u, dv = vo - v;
    if (du > cols / 2.0) du -= cols;
    else if (du < -cols / 2.0) du += cols;
    if (fabs(du) > 100.0 || fabs(dv) > 100.0) {
        r[0] = 100.0; r[1] = 100.0;
        return 0;
    }
    r[0] = Lw[0] * du;
    r[1] = Lw[2] * du + Lw[3] * dv;
    tail = true;
    return 0;
}

// The compressed Jacobian of factor_eval_ap at a point whose residual was linearised with Jacobian scale asc
// (the Huber / Corrector scale, 0 when the Jacobian was zero: outlier, degenerate or out-of-range residual):
// A = asc Jw R_cb_raw and Pb, recomputed from the point and the pose cache at the linearisation point (pcl:
// Rbw(9) tbw(3) Rcw(9) tcw(3), i.e. pose_cache_one's output from offset 12) with factor_eval_ap's own
// operations (factor_ap_tail).  The window solver's phase kernels keep only r and asc per observation
// (24 B instead of 88 B) and rebuild A / Pb where they are used.
__device__ __forceinline__ void factor_ap_at(const double* pcl, const double* Rcb_raw, const double* Pw, double cols,
                                             double rows, const double* Lw, double asc, double* A, double* Pb) {
    if (asc == 0.0) {
#pragma unroll
        for (int i = 0; i < 6; ++i) A[i] = 0.0;
#pragma unroll
        for (int i = 0; i < 3; ++i) Pb[i] = 0.0;
        return;
    }
    const double* Rbw = pcl;
    const double* tbw = pcl + 9;
    const double* Rcw = pcl + 12;
    const double* tcw = pcl + 21;
    double Pc[3];
    m3vec(Rcw, Pw, Pc);
    Pc[0] += tcw[0]; Pc[1] += tcw[1]; Pc[2] += tcw[2];
    const double L = nrm3(Pc);
    const double iL = 1.0 / L;
    factor_ap_tail(Pc[0], Pc[1], Pc[2], L, iL, Rbw, tbw, Pw, Rcb_raw, cols, rows, Lw, A, Pb);
#pragma unroll
    for (int i = 0; i < 6; ++i) A[i] *= asc;
}

// compute_chi_square (Factors.cpp:212-265, 544-612), unweighted e^T Info e
__device__ __forceinline__ double factor_chi2(const double* pc, const double* Pw, double uo, double vo, double cols,
                                              double rows, const double* info, bool outlier, bool is_pnp) {
    if (outlier && !is_pnp) return 0.0;
    const double* Rcw = pc + 24;
    const double* tcw = pc + 33;
    double Pc[3];
    m3vec(Rcw, Pw, Pc);
    Pc[0] += tcw[0]; Pc[1] += tcw[1]; Pc[2] += tcw[2];
    double L = nrm3(Pc);
    if (L < 1e-10) return is_pnp ? DBL_MAX : 1000.0;
    double theta = atan2(Pc[0], Pc[2]);
    double phi = -asin(Pc[1] / L);
    double u = cols * (0.5 + theta / (2.0 * M_PI));
    double v = rows * (0.5 - phi / M_PI);
    double du = uo - u, dv = vo - v;
    if (du > cols / 2.0) du -= cols;
    else if (du < -cols / 2.0) du += cols;
    return du * (info[0] * du + info[1] * dv) + dv * (info[2] * du + info[3] * dv);
}


}  // namespace vio360
