"""tri_oracle.py — TEST INFRASTRUCTURE ONLY (parity checker + timed CPU baseline, never shipped).

numpy restatement of Estimator::TriangulateSinglePoint (src/processing/Estimator.cpp:1082-1137) and
of the reprojection angle errors TriangulateNewMapPoints computes per new point (:1233-1248):
A is built in f32 with the reference's expressions (b(0)·T.row(2) − b(2)·T.row(0), ...), the null
vector comes from LAPACK's SVD in f64 (numpy.linalg.svd) — the reference runs Eigen's f32 JacobiSVD
(Eigen is not in /root/reference nor in this image, so bitwise parity with the reference binary is
unpinned; the null vector is unique up to sign for a rank-3 A).  Pinned by exact synthetic geometry
(tests/test_tri_oracle.py): noise-free bearings of known points recover the points to f32 rounding.
"""
import math

import numpy as np

F32 = np.float32


def build_A(T1, T2, b1, b2):
    """(n,4,4) f32 A rows exactly as Estimator.cpp:1098-1101 (f32 elementwise, no contraction)."""
    b1 = np.asarray(b1, F32)
    b2 = np.asarray(b2, F32)
    A = np.empty(b1.shape[:-1] + (4, 4), F32)
    A[..., 0, :] = b1[..., 0:1] * T1[..., 2, :] - b1[..., 2:3] * T1[..., 0, :]
    A[..., 1, :] = b1[..., 1:2] * T1[..., 2, :] - b1[..., 2:3] * T1[..., 1, :]
    A[..., 2, :] = b2[..., 0:1] * T2[..., 2, :] - b2[..., 2:3] * T2[..., 0, :]
    A[..., 3, :] = b2[..., 1:2] * T2[..., 2, :] - b2[..., 2:3] * T2[..., 1, :]
    return A


def reproj_px(T, b, X, width):
    """Estimator.cpp:1233-1248 in f32: acos(min(1, |b·normalize(T·[X;1])|))·width / (2π)."""
    T = np.asarray(T, F32)
    pc = ((T[..., :, 0] * X[..., 0:1] + T[..., :, 1] * X[..., 1:2]) + T[..., :, 2] * X[..., 2:3]) + T[..., :, 3]
    pc = pc[..., :3]
    nrm = np.sqrt((pc[..., 0] * pc[..., 0] + pc[..., 1] * pc[..., 1]) + pc[..., 2] * pc[..., 2])
    safe = np.where(nrm > 0, nrm, F32(1))
    u = pc / safe[..., None]
    dot = np.where(nrm > 0, (b[..., 0] * u[..., 0] + b[..., 1] * u[..., 1]) + b[..., 2] * u[..., 2], F32(0))
    ang = np.arccos(np.minimum(F32(1), np.abs(dot))).astype(F32)
    return ((ang * F32(width)).astype(np.float64) / (2.0 * math.pi)).astype(F32)


def triangulate(T_cw, pairs, bearings, width):
    """Same contract as vio_triangulate: returns (points (n,3) f32, valid (n,) u8, pixel_err (n,2) f32)."""
    T_cw = np.asarray(T_cw, F32).reshape(-1, 4, 4)
    pairs = np.asarray(pairs, np.int32).reshape(-1, 2)
    bearings = np.asarray(bearings, F32).reshape(-1, 6)
    n = len(pairs)
    T1, T2 = T_cw[pairs[:, 0]], T_cw[pairs[:, 1]]
    b1, b2 = bearings[:, :3], bearings[:, 3:]
    A = build_A(T1, T2, b1, b2).astype(np.float64)
    X = np.zeros((n, 3), F32)
    valid = np.zeros(n, np.uint8)
    err = np.zeros((n, 2), F32)
    if n == 0:
        return X, valid, err
    _, _, Vt = np.linalg.svd(A)
    v = Vt[:, 3, :]
    ok = np.abs(v[:, 3]) >= 1e-10
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        P = (v[:, :3] / np.where(ok, v[:, 3], 1.0)[:, None]).astype(F32)
    ok &= np.isfinite(P).all(1)
    X[ok] = P[ok]
    valid[ok] = 1
    e1 = reproj_px(T1, b1, X, width)
    e2 = reproj_px(T2, b2, X, width)
    err[:, 0] = np.where(ok, e1, 0)
    err[:, 1] = np.where(ok, e2, 0)
    return X, valid, err
