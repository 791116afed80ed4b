"""Generate tests/golden/factor_golden.npz — golden vectors for the ERP reprojection factor.

Independent numpy restatement of BAFactor::Evaluate / PnPFactor::Evaluate
(src/optimization/Factors.cpp:327-542, :33-210) and BAFactor::compute_chi_square (:544-612),
built on LAPACK SVD for the SO3d(Matrix3d) projection (src/util/LieUtils.cpp:275-288) instead of
the C oracle's Jacobi eigen-solver, so the two restatements share no code.  The reference itself
cannot be compiled in this image (no Eigen / OpenCV), so these vectors pin the C
oracle and the HIP kernels against a second reading of the reference source, not against the
reference binary ("parity unpinned" against the binary).

Run:  python tests/golden/gen_factor_golden.py   (deterministic, seed fixed)
"""
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def so3d(M):
    """SO3d(const Matrix3d&): U V^T, flip U col 2 if det < 0 (LieUtils.cpp:275-288)."""
    U, _, Vt = np.linalg.svd(M)
    R = U @ Vt
    if np.linalg.det(R) < 0:
        U[:, 2] *= -1
        R = U @ Vt
    return R


def hat(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]], dtype=np.float64)


def so3_exp(w):
    """SO3d::Exp (LieUtils.cpp:203-219)."""
    th = np.linalg.norm(w)
    if th < 1e-10:
        return so3d(np.eye(3) + hat(w))
    K = hat(w / th)
    return so3d(np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K)


def se3_exp(xi):
    """SE3d::exp (LieUtils.cpp:305-333): xi = [rho, phi]."""
    rho, phi = xi[:3], xi[3:]
    R = so3_exp(phi)
    th = np.linalg.norm(phi)
    if th < 1e-10:
        return R, rho.copy()
    P = hat(phi)
    V = np.eye(3) + (1 - math.cos(th)) / th**2 * P + (th - math.sin(th)) / th**3 * P @ P
    return R, V @ rho


def compose(A, B):
    """SE3d operator* (LieUtils.h:268-271)."""
    return so3d(A[0] @ B[0]), A[1] + A[0] @ B[1]


def inverse(A):
    """SE3d::inverse (LieUtils.h:279-282)."""
    Ri = so3d(A[0].T)
    return Ri, Ri @ (-A[1])


def factor(T_init, T_cb, delta, Pw, obs, cols, rows, outlier=False, is_pnp=False):
    """Returns (ok, r[2], Jp[2x6], Jl[2x3]) for identity information."""
    z12, z6 = np.zeros((2, 6)), np.zeros((2, 3))
    if outlier:
        return True, np.array([640.0, 480.0]), z12, z6
    Twb = compose((so3d(T_init[:3, :3]), T_init[:3, 3]), se3_exp(delta))
    Tbw = inverse(Twb)
    Tcw = compose((so3d(T_cb[:3, :3]), T_cb[:3, 3]), Tbw)
    Pc = Tcw[0] @ Pw + Tcw[1]
    x, y, z = Pc
    L = np.linalg.norm(Pc)
    if L < 1e-10:
        if is_pnp:
            return False, np.zeros(2), z12, z6
        return True, np.array([640.0, 360.0]), z12, z6
    theta = math.atan2(x, z)
    phi = -math.asin(y / L)
    u = cols * (0.5 + theta / (2 * math.pi))
    v = rows * (0.5 - phi / math.pi)
    du, dv = obs[0] - u, obs[1] - v
    if du > cols / 2:
        du -= cols
    elif du < -cols / 2:
        du += cols
    if abs(du) > 100 or abs(dv) > 100:
        return True, np.array([100.0, 100.0]), z12, z6
    r = np.array([du, dv])
    xz2 = x * x + z * z
    if xz2 < 1e-10 or L * L < 1e-10:
        return True, r, z12, z6
    xzn = math.sqrt(xz2)
    Jc = np.array([[-cols / (2 * math.pi) * z / xz2, 0.0, cols / (2 * math.pi) * x / xz2],
                   [rows / math.pi * x * y / (L * L * xzn), -rows / math.pi * xzn / (L * L),
                    rows / math.pi * y * z / (L * L * xzn)]])
    Rcb = T_cb[:3, :3]  # m_Tcb.block<3,3> used verbatim (not projected) in the Jacobians
    Pb = Tbw[0] @ Pw + Tbw[1]
    Jp = Jc @ np.hstack([-Rcb, Rcb @ hat(Pb)])
    Jl = Jc @ (Rcb @ Tbw[0])
    return True, r, Jp, Jl


def chi2(T_init, T_cb, delta, Pw, obs, cols, rows, outlier=False, is_pnp=False):
    """compute_chi_square with identity information (Factors.cpp:212-265, 544-612)."""
    if outlier and not is_pnp:
        return 0.0
    Twb = compose((so3d(T_init[:3, :3]), T_init[:3, 3]), se3_exp(delta))
    Tcw = compose((so3d(T_cb[:3, :3]), T_cb[:3, 3]), inverse(Twb))
    Pc = Tcw[0] @ Pw + Tcw[1]
    L = np.linalg.norm(Pc)
    if L < 1e-10:
        return np.finfo(np.float64).max if is_pnp else 1000.0
    u = cols * (0.5 + math.atan2(Pc[0], Pc[2]) / (2 * math.pi))
    v = rows * (0.5 + math.asin(Pc[1] / L) / math.pi)
    du, dv = obs[0] - u, obs[1] - v
    if du > cols / 2:
        du -= cols
    elif du < -cols / 2:
        du += cols
    return du * du + dv * dv


def rand_rot(rng, deg):
    w = rng.normal(0, math.radians(deg), 3)
    th = np.linalg.norm(w)
    K = hat(w / th)
    return np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K


def main():
    rng = np.random.default_rng(1205)
    cols, rows = 960.0, 480.0
    T_bc = np.array([[-0.0013741, -0.99974421, -0.02257504, 0.01065397],
                     [-0.02183404, -0.02253969, 0.9995075, 0.00614827],
                     [-0.99976066, 0.00186632, -0.02179749, 0.01690583],
                     [0, 0, 0, 1]], np.float32)
    T_cb = np.linalg.inv(T_bc.astype(np.float64)).astype(np.float32).astype(np.float64)
    cases = []
    n = 96
    for i in range(n):
        T = np.eye(4)
        T[:3, :3] = rand_rot(rng, 40.0)
        T[:3, 3] = rng.normal(0, 1.0, 3)
        T = T.astype(np.float32).astype(np.float64)  # f32 Frame storage -> raw (non-orthonormal) f64
        delta = rng.normal(0, 0.02, 6) if i % 4 else np.zeros(6)
        Tcw_R = T_cb[:3, :3] @ T[:3, :3].T
        # landmark in front of / around the camera at 2..10 m
        lon, lat = rng.uniform(-math.pi, math.pi), rng.uniform(-1.2, 1.2)
        b = np.array([math.cos(lat) * math.sin(lon), -math.sin(lat), math.cos(lat) * math.cos(lon)])
        Pc = b * rng.uniform(2, 10)
        twc = T[:3, :3] @ (-T_cb[:3, :3].T @ T_cb[:3, 3]) + T[:3, 3]
        Pw = Tcw_R.T @ Pc + twc
        Twb = compose((so3d(T[:3, :3]), T[:3, 3]), se3_exp(delta))
        Tcw = compose((so3d(T_cb[:3, :3]), T_cb[:3, 3]), inverse(Twb))
        Pc2 = Tcw[0] @ Pw + Tcw[1]
        u = cols * (0.5 + math.atan2(Pc2[0], Pc2[2]) / (2 * math.pi))
        v = rows * (0.5 + math.asin(Pc2[1] / np.linalg.norm(Pc2)) / math.pi)
        obs = np.array([u, v]) + rng.normal(0, 2.0, 2)
        kind = i % 12
        outlier = False
        if kind == 1:          # |du| > 100 branch
            obs[0] += 150.0
        elif kind == 2:        # horizontal wrap: observation on the other side of the seam
            obs[0] = obs[0] - cols if obs[0] > cols / 2 else obs[0] + cols
        elif kind == 3:        # outlier flag
            outlier = True
        elif kind == 4:        # |Pc| < 1e-10: landmark at the camera centre
            Pw = Tcw[0].T @ (-Tcw[1])
        elif kind == 5:        # x^2 + z^2 < 1e-10: landmark (almost) straight above the camera -> J zeroed
            Pc5 = np.array([3e-6, -3.0, 4e-6])
            Pw = Tcw[0].T @ (Pc5 - Tcw[1])
            u5 = cols * (0.5 + math.atan2(Pc5[0], Pc5[2]) / (2 * math.pi))
            v5 = rows * (0.5 + math.asin(Pc5[1] / np.linalg.norm(Pc5)) / math.pi)
            obs = np.array([u5, v5]) + rng.normal(0, 2.0, 2)
        obs = obs.astype(np.float32).astype(np.float64)
        for is_pnp in (False, True):
            ok, r, Jp, Jl = factor(T, T_cb, delta, Pw, obs, cols, rows, outlier, is_pnp)
            c2 = chi2(T, T_cb, delta, Pw, obs, cols, rows, outlier, is_pnp)
            cases.append(dict(T=T, delta=delta, Pw=Pw, obs=obs, outlier=outlier, is_pnp=is_pnp, ok=ok, r=r,
                              Jp=Jp, Jl=Jl, chi2=c2))
    out = {k: np.array([c[k] for c in cases]) for k in cases[0]}
    out["T_cb"] = T_cb
    out["cols"] = np.array(cols)
    out["rows"] = np.array(rows)
    np.savez_compressed(os.path.join(HERE, "factor_golden.npz"), **out)
    print("wrote", len(cases), "cases")


if __name__ == "__main__":
    main()
