"""Loader for the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    so = os.path.join(ORACLE_DIR, "liboracle.so")
    if not os.path.exists(so):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    L = C.CDLL(so)
    L.oracle_ba_solve.argtypes = [C.c_void_p, C.c_void_p]
    vp = C.c_void_p
    L.oracle_imu_preintegrate.argtypes = [vp, C.c_int, vp, vp, C.c_int, vp, vp, vp, vp, vp, vp]
    L.oracle_set_threads.argtypes = [C.c_int]
    _lib = L
    return L


def ba_solve(vio, prob):
    """Run the oracle on a vio.BaProblem; returns the same result dict as the HIP path."""
    L = load()
    O = vio.BaOutput(prob.K, prob.L, prob.N)
    rc = L.oracle_ba_solve(C.byref(prob.c), C.byref(O.c))
    if rc != 0:
        raise RuntimeError(f"oracle_ba_solve rc={rc}")
    return O.result()


def imu_preintegrate(vio, samples, t_start, t_end, gyro_bias=None, accel_bias=None, noise=None):
    """oracle/imu_oracle.c through the same marshalling as Context.imu_preintegrate."""
    L = load()

    def check(rc, what):
        if rc != 0:
            raise RuntimeError(f"oracle {what} rc={rc}")
    return vio._imu_call(L.oracle_imu_preintegrate, check, samples, t_start, t_end, gyro_bias, accel_bias, noise)


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def klt_track(prev, curr, pts, params):
    L = load()
    prev = np.ascontiguousarray(prev, np.uint8)
    curr = np.ascontiguousarray(curr, np.uint8)
    H, W = prev.shape
    pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 2)
    n = len(pts)
    nxt = np.zeros((n, 2), np.float32)
    st = np.zeros(n, np.uint8)
    err = np.zeros(n, np.float32)
    rc = L.oracle_klt_track(_p(prev), _p(curr), W, H, W, _p(pts), n, _p(nxt), _p(st), _p(err), C.byref(params))
    assert rc == 0
    return nxt, st, err


def gftt(img, mask, max_corners, quality, min_dist):
    L = load()
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape
    m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    cap = max_corners if max_corners > 0 else W * H
    out = np.zeros((cap, 2), np.float32)
    n = C.c_int()
    rc = L.oracle_gftt(_p(img), _p(m) if m is not None else None, W, H, W, int(max_corners), C.c_double(quality),
                       C.c_double(min_dist), _p(out), C.byref(n))
    assert rc == 0
    return out[: n.value].copy()


def rot_ransac(p0, p1, W, H, samples, thresh):
    L = load()
    p0 = np.ascontiguousarray(p0, np.float32).reshape(-1, 2)
    p1 = np.ascontiguousarray(p1, np.float32).reshape(-1, 2)
    samples = np.ascontiguousarray(samples, np.int32).reshape(-1)
    n = len(p0)
    mask = np.zeros(n, np.uint8)
    nin = C.c_int()
    rc = L.oracle_rot_ransac(_p(p0), _p(p1), n, W, H, _p(samples), len(samples) // 3, C.c_float(thresh), _p(mask),
                             C.byref(nin))
    assert rc == 0
    return mask, nin.value


def min_eig_map(img):
    L = load()
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape
    eig = np.zeros((H, W), np.float32)
    L.oracle_min_eig_map(_p(img), W, H, W, _p(eig))
    return eig


def pyr_down(img):
    L = load()
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape
    out = np.zeros(((H + 1) // 2, (W + 1) // 2), np.uint8)
    L.oracle_pyr_down(_p(img), W, H, W, _p(out), out.shape[1])
    return out


def pixel_to_bearing(u, v, W, H):
    L = load()
    b = np.zeros(3, np.float32)
    L.oracle_pixel_to_bearing(C.c_float(u), C.c_float(v), W, H, _p(b))
    return b


def imu_init(vio, prob):
    """oracle_imu_init on an abi.ImuInitProblem; the same result dict as Context.imu_init."""
    L = load()
    out = vio.abi.ImuInitResult(prob.F)
    rc = L.oracle_imu_init(C.byref(prob.c), C.byref(out.c))
    if rc != 0:
        raise RuntimeError(f"oracle_imu_init rc={rc}")
    return out.result()


def mono_init(vio, b1, b2, samples, params):
    """oracle/init_oracle.c (TryMonocularInitialization restated) with the C-ABI's structs."""
    L = load()
    b1 = np.ascontiguousarray(b1, np.float32).reshape(-1, 3)
    b2 = np.ascontiguousarray(b2, np.float32).reshape(-1, 3)
    S = np.ascontiguousarray(samples, np.int32).reshape(-1, 8)
    n = len(b1)
    R = vio.abi.VioMonoInitResult()
    M = np.zeros(max(n, 1), np.uint8)
    X = np.zeros((max(n, 1), 3), np.float32)
    L.oracle_mono_init.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_void_p]
    L.oracle_mono_init(_p(b1), _p(b2), n, _p(S), C.byref(params), C.byref(R), _p(M), _p(X))
    return vio.abi.mono_init_result_dict(R), M[:n], X[:n]
