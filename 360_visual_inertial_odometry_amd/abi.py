"""ctypes mirror of include/vio360.h (the C-ABI boundary).

Only plain C types cross the boundary; the structures below must stay byte-identical to the
header (checked by tests/test_abi.py against offsetof values compiled from the header).
"""
import ctypes as C

import numpy as np

VIO_BA_LOCAL, VIO_BA_FULL, VIO_BA_VI, VIO_PNP = 0, 1, 2, 3
VIO_TERM_CONVERGENCE, VIO_TERM_NO_CONVERGENCE, VIO_TERM_FAILURE = 0, 1, 2

_u8p = C.POINTER(C.c_uint8)
_i32p = C.POINTER(C.c_int32)
_f32p = C.POINTER(C.c_float)
_f64p = C.POINTER(C.c_double)


class VioPose(C.Structure):
    _fields_ = [("R", C.c_double * 9), ("t", C.c_double * 3)]


class VioPreint(C.Structure):
    _fields_ = [
        ("delta_R", C.c_float * 9), ("delta_V", C.c_float * 3), ("delta_P", C.c_float * 3),
        ("J_Rg", C.c_float * 9), ("J_Vg", C.c_float * 9), ("J_Va", C.c_float * 9),
        ("J_Pg", C.c_float * 9), ("J_Pa", C.c_float * 9),
        ("cov9", C.c_float * 81), ("gyro_bias", C.c_float * 3), ("accel_bias", C.c_float * 3),
        ("_pad", C.c_float * 2), ("dt_total", C.c_double),
    ]


class VioBaProblem(C.Structure):
    _fields_ = [
        ("variant", C.c_int32), ("num_kf", C.c_int32), ("num_lm", C.c_int32), ("num_obs", C.c_int32),
        ("cols", C.c_double), ("rows", C.c_double), ("huber_delta", C.c_double),
        ("info", C.c_double * 4), ("chi2_threshold", C.c_double),
        ("T_cb", C.POINTER(VioPose)), ("T_wb_init", C.POINTER(VioPose)),
        ("kf_const", _u8p), ("lm_const", _u8p), ("lm_marg", _u8p),
        ("lm_xyz", _f64p), ("obs_kf", _i32p), ("obs_lm", _i32p), ("obs_uv", _f32p),
        ("preint", C.POINTER(VioPreint)), ("preint_valid", _u8p), ("vel", _f64p),
        ("bg", C.c_double * 3), ("ba", C.c_double * 3), ("gravity", C.c_double * 3),
        ("max_iterations", C.c_int32), ("fixed_iterations", C.c_int32),
        ("num_rounds", C.c_int32), ("_pad0", C.c_int32),
    ]


class VioBaSummary(C.Structure):
    _fields_ = [
        ("success", C.c_int32), ("termination", C.c_int32), ("iterations", C.c_int32),
        ("num_successful_steps", C.c_int32), ("num_unsuccessful_steps", C.c_int32),
        ("num_inliers", C.c_int32), ("num_outliers", C.c_int32), ("num_bad_lm", C.c_int32),
        ("initial_cost", C.c_double), ("final_cost", C.c_double), ("fixed_cost", C.c_double),
        ("_pad1", C.c_double),
    ]


class VioBaIteration(C.Structure):
    """Solver::Summary::iterations entry (ceres IterationSummary fields the solver sets)."""
    _fields_ = [
        ("iteration", C.c_int32), ("step_is_valid", C.c_int32), ("step_is_successful", C.c_int32),
        ("_pad", C.c_int32), ("cost", C.c_double), ("cost_change", C.c_double),
        ("gradient_max_norm", C.c_double), ("step_norm", C.c_double), ("relative_decrease", C.c_double),
        ("trust_region_radius", C.c_double), ("model_cost_change", C.c_double),
    ]


TRACE_FIELDS = ("iteration", "step_is_valid", "step_is_successful", "cost", "cost_change", "gradient_max_norm",
                "step_norm", "relative_decrease", "trust_region_radius", "model_cost_change")


class VioBaOutput(C.Structure):
    _fields_ = [
        ("T_wb", C.POINTER(VioPose)), ("lm_xyz", _f64p), ("obs_chi2", _f64p), ("obs_outlier", _u8p),
        ("lm_bad", _u8p), ("vel", _f64p), ("bg", _f64p), ("ba", _f64p),
        ("summary", C.POINTER(VioBaSummary)),
        ("trace", C.POINTER(VioBaIteration)), ("trace_cap", C.c_int32), ("_pad2", C.c_int32),
    ]


class ErpKltParams(C.Structure):
    _fields_ = [("win", C.c_int32), ("max_level", C.c_int32), ("max_iters", C.c_int32),
                ("epsilon", C.c_float), ("min_eig_threshold", C.c_float), ("_pad", C.c_int32)]


class ErpTrackerParams(C.Structure):
    _fields_ = [("ransac_iters", C.c_int32), ("ransac_thresh_rad", C.c_float), ("ransac_seed", C.c_uint32),
                ("max_corners", C.c_int32), ("quality", C.c_double), ("min_dist", C.c_double),
                ("boundary_margin", C.c_int32), ("polar_ratio", C.c_float)]


class ErpFrontendParams(C.Structure):
    _fields_ = [("max_features", C.c_int32), ("min_distance", C.c_float), ("quality_level", C.c_float),
                ("boundary_margin", C.c_int32), ("grid_cols", C.c_int32), ("grid_rows", C.c_int32),
                ("max_features_per_grid", C.c_int32), ("remove_clustered", C.c_int32),
                ("clustered_std_ratio", C.c_float), ("ransac_seed", C.c_uint32)]


def default_frontend_params(seed=0):
    """config/default_config.yaml values the tracker reads (feature_detection.*, camera.boundary_margin,
    visualization.highlight_clustered_grid / clustered_std_ratio)."""
    return ErpFrontendParams(1000, 30.0, 0.01, 20, 20, 10, 10, 1, 0.25, seed)


def default_klt_params():
    """FeatureTracker's hard-coded LK settings (src/processing/FeatureTracker.cpp:33-35,240)."""
    return ErpKltParams(21, 3, 30, 0.01, 0.01, 0)


def default_tracker_params(max_corners=300, seed=0):
    """FeatureTracker's settings (src/processing/FeatureTracker.cpp:36-38, config feature_detection.*;
    quality_level is a float member, so 0.01f reaches OpenCV as a double)."""
    thr = float(np.float32(np.float64(np.float32(2.0)) * np.pi / np.float64(np.float32(180.0))))
    return ErpTrackerParams(1000, thr, seed, max_corners, float(np.float32(0.01)), 30.0, 20, 0.15)


def _ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype)) if a is not None else None


def poses_to_c(T):
    """(K,4,4) or (K,3,4) float array -> ctypes array of VioPose (f64)."""
    T = np.asarray(T, dtype=np.float64)
    arr = (VioPose * len(T))()
    for k in range(len(T)):
        arr[k].R[:] = T[k, :3, :3].reshape(-1).tolist()
        arr[k].t[:] = T[k, :3, 3].tolist()
    return arr


def poses_from_c(arr, K):
    out = np.zeros((K, 4, 4))
    for k in range(K):
        out[k, :3, :3] = np.array(arr[k].R[:]).reshape(3, 3)
        out[k, :3, 3] = arr[k].t[:]
        out[k, 3, 3] = 1.0
    return out


def preints_to_c(preints):
    """list (len K, entry 0 may be None) of dicts -> (VioPreint array, valid u8 array)."""
    K = len(preints)
    arr = (VioPreint * K)()
    valid = np.zeros(K, np.uint8)
    for k, p in enumerate(preints):
        if p is None:
            continue
        valid[k] = 1
        e = arr[k]
        e.delta_R[:] = np.asarray(p["delta_R"], np.float32).reshape(-1).tolist()
        e.delta_V[:] = np.asarray(p["delta_V"], np.float32).tolist()
        e.delta_P[:] = np.asarray(p["delta_P"], np.float32).tolist()
        for nm in ("J_Rg", "J_Vg", "J_Va", "J_Pg", "J_Pa"):
            getattr(e, nm)[:] = np.asarray(p[nm], np.float32).reshape(-1).tolist()
        e.cov9[:] = np.asarray(p["cov"], np.float32)[:9, :9].reshape(-1).tolist()
        e.gyro_bias[:] = np.asarray(p["gyro_bias"], np.float32).tolist()
        e.accel_bias[:] = np.asarray(p["accel_bias"], np.float32).tolist()
        e.dt_total = float(p["dt_total"])
    return arr, valid


class BaProblem:
    """Owns numpy buffers + the ctypes struct pointing at them (keeps everything alive)."""

    def __init__(self, window, variant=VIO_BA_LOCAL, max_iterations=50, fixed_iterations=0,
                 chi2_threshold=None, num_rounds=4, huber_delta=1.0):
        w = window
        self.K = int(len(w["T_wb_init"]))
        self.L = int(len(w["lm_xyz"]))
        self.N = int(len(w["obs_kf"]))
        self.variant = variant
        self.T_cb = poses_to_c(w["T_cb"] if np.ndim(w["T_cb"]) == 3 else np.repeat(np.asarray(w["T_cb"])[None], self.K, 0))
        self.T_wb_init = poses_to_c(w["T_wb_init"])
        self.kf_const = np.ascontiguousarray(w["kf_const"], np.uint8)
        self.lm_const = np.ascontiguousarray(w["lm_const"], np.uint8)
        self.lm_marg = np.ascontiguousarray(w.get("lm_marg", np.zeros(self.L, np.uint8)), np.uint8)
        self.lm_xyz = np.ascontiguousarray(w["lm_xyz"], np.float64).reshape(-1)
        self.obs_kf = np.ascontiguousarray(w["obs_kf"], np.int32)
        self.obs_lm = np.ascontiguousarray(w["obs_lm"], np.int32)
        self.obs_uv = np.ascontiguousarray(w["obs_uv"], np.float32).reshape(-1)
        p = VioBaProblem()
        p.variant = variant
        p.num_kf, p.num_lm, p.num_obs = self.K, self.L, self.N
        p.cols, p.rows = float(w["cols"]), float(w["rows"])
        p.huber_delta = huber_delta
        p.info[:] = [1.0, 0.0, 0.0, 1.0]
        if chi2_threshold is None:
            chi2_threshold = 5.99146 if variant == VIO_BA_LOCAL else 5.991
        p.chi2_threshold = chi2_threshold
        p.T_cb = C.cast(self.T_cb, C.POINTER(VioPose))
        p.T_wb_init = C.cast(self.T_wb_init, C.POINTER(VioPose))
        p.kf_const = _ptr(self.kf_const, C.c_uint8)
        p.lm_const = _ptr(self.lm_const, C.c_uint8)
        p.lm_marg = _ptr(self.lm_marg, C.c_uint8)
        p.lm_xyz = _ptr(self.lm_xyz, C.c_double)
        p.obs_kf = _ptr(self.obs_kf, C.c_int32)
        p.obs_lm = _ptr(self.obs_lm, C.c_int32)
        p.obs_uv = _ptr(self.obs_uv, C.c_float)
        if variant == VIO_BA_VI:
            self.preint, self.preint_valid = preints_to_c(w["preint"])
            self.vel = np.ascontiguousarray(w["vel"], np.float64).reshape(-1)
            p.preint = C.cast(self.preint, C.POINTER(VioPreint))
            p.preint_valid = _ptr(self.preint_valid, C.c_uint8)
            p.vel = _ptr(self.vel, C.c_double)
            p.bg[:] = list(np.asarray(w.get("bg", np.zeros(3)), np.float64))
            p.ba[:] = list(np.asarray(w.get("ba", np.zeros(3)), np.float64))
            p.gravity[:] = list(np.asarray(w["gravity"], np.float64))
        p.max_iterations = max_iterations
        p.fixed_iterations = fixed_iterations
        p.num_rounds = num_rounds
        self.c = p


class BaOutput:
    def __init__(self, K, L, N, trace_cap=256):
        self.K, self.L, self.N = K, L, N
        self.T_wb = (VioPose * K)()
        self.lm_xyz = np.zeros(3 * max(L, 1))
        self.obs_chi2 = np.zeros(max(N, 1))
        self.obs_outlier = np.zeros(max(N, 1), np.uint8)
        self.lm_bad = np.zeros(max(L, 1), np.uint8)
        self.vel = np.zeros(3 * K)
        self.bg = np.zeros(3)
        self.ba = np.zeros(3)
        self.summary = VioBaSummary()
        o = VioBaOutput()
        o.T_wb = C.cast(self.T_wb, C.POINTER(VioPose))
        o.lm_xyz = _ptr(self.lm_xyz, C.c_double)
        o.obs_chi2 = _ptr(self.obs_chi2, C.c_double)
        o.obs_outlier = _ptr(self.obs_outlier, C.c_uint8)
        o.lm_bad = _ptr(self.lm_bad, C.c_uint8)
        o.vel = _ptr(self.vel, C.c_double)
        o.bg = _ptr(self.bg, C.c_double)
        o.ba = _ptr(self.ba, C.c_double)
        o.summary = C.pointer(self.summary)
        self.trace = (VioBaIteration * max(trace_cap, 1))()
        o.trace = C.cast(self.trace, C.POINTER(VioBaIteration))
        o.trace_cap = trace_cap
        self.c = o

    def result(self):
        s = self.summary
        return {
            "T_wb": poses_from_c(self.T_wb, self.K),
            "lm_xyz": self.lm_xyz[: 3 * self.L].reshape(-1, 3).copy(),
            "obs_chi2": self.obs_chi2[: self.N].copy(),
            "obs_outlier": self.obs_outlier[: self.N].copy(),
            "lm_bad": self.lm_bad[: self.L].copy(),
            "vel": self.vel.reshape(-1, 3).copy(),
            "bg": self.bg.copy(),
            "ba": self.ba.copy(),
            "success": s.success, "termination": s.termination, "iterations": s.iterations,
            "num_successful_steps": s.num_successful_steps,
            "num_unsuccessful_steps": s.num_unsuccessful_steps,
            "num_inliers": s.num_inliers, "num_outliers": s.num_outliers, "num_bad_lm": s.num_bad_lm,
            "initial_cost": s.initial_cost, "final_cost": s.final_cost, "fixed_cost": s.fixed_cost,
            "trace": self.trace_dict(),
        }

    def trace_dict(self):
        """Summary::iterations as a dict of numpy arrays (one entry per recorded iteration)."""
        n = min(max(self.summary.iterations, 0), self.c.trace_cap)
        return {f: np.array([getattr(self.trace[i], f) for i in range(n)]) for f in TRACE_FIELDS}


# ---------------------------------------------------------------------------------------------
# IMU preintegration (vio_imu_preintegrate)
class VioImuData(C.Structure):
    """IMUData (src/processing/Estimator.h:32-36)."""
    _fields_ = [("timestamp", C.c_double), ("ax", C.c_float), ("ay", C.c_float), ("az", C.c_float),
                ("gx", C.c_float), ("gy", C.c_float), ("gz", C.c_float)]


class VioImuNoise(C.Structure):
    _fields_ = [("gyro_noise", C.c_float), ("accel_noise", C.c_float), ("gyro_bias_noise", C.c_float),
                ("accel_bias_noise", C.c_float)]


IMU_DTYPE = np.dtype({"names": ["timestamp", "ax", "ay", "az", "gx", "gy", "gz"],
                      "formats": ["<f8"] + ["<f4"] * 6, "offsets": [0, 8, 12, 16, 20, 24, 28],
                      "itemsize": C.sizeof(VioImuData)})
PREINT_FIELDS = (("delta_R", (3, 3)), ("delta_V", (3,)), ("delta_P", (3,)), ("J_Rg", (3, 3)), ("J_Vg", (3, 3)),
                 ("J_Va", (3, 3)), ("J_Pg", (3, 3)), ("J_Pa", (3, 3)), ("cov9", (9, 9)), ("gyro_bias", (3,)),
                 ("accel_bias", (3,)))


def imu_array(samples):
    """(M, 7) array of [t, ax, ay, az, gx, gy, gz] (synth.imu_samples layout) -> vio_imu_data records."""
    s = np.asarray(samples, dtype=np.float64).reshape(-1, 7)
    out = np.zeros(len(s), IMU_DTYPE)
    out["timestamp"] = s[:, 0]
    for k, name in enumerate(("ax", "ay", "az", "gx", "gy", "gz")):
        out[name] = s[:, 1 + k].astype(np.float32)
    return out


def imu_noise(noise=None):
    """VioImuNoise from a (gyro, accel, gyro_bias, accel_bias) tuple; None = the reference defaults."""
    if noise is None:
        noise = (1.0e-4, 1.0e-3, 1.0e-6, 1.0e-5)
    return VioImuNoise(*[float(x) for x in noise])


def preint_records(out):
    """(VioPreint * n) -> dict of stacked numpy arrays (n, ...) keyed by the IMUPreintegration fields."""
    n = len(out)
    flat = np.frombuffer(out, dtype=np.uint8).reshape(n, C.sizeof(VioPreint)) if n else np.zeros((0, C.sizeof(VioPreint)), np.uint8)
    res = {}
    for name, shape in PREINT_FIELDS:
        off = getattr(VioPreint, name).offset
        cnt = int(np.prod(shape))
        res[name] = flat[:, off:off + 4 * cnt].copy().view(np.float32).reshape((n,) + shape)
    off = VioPreint.dt_total.offset
    res["dt_total"] = flat[:, off:off + 8].copy().view(np.float64).reshape(n)
    return res



# ---------------------------------------------------------------------------------------------
# Problem assembly / write-back on the flat Frame / Feature / MapPoint graph (vio_ba_gather,
# vio_ba_write_back; Optimizer.cpp gather filters and write-back rules)
VIO_GATHER_OK, VIO_GATHER_FEW_FRAMES, VIO_GATHER_NO_MAPPOINTS, VIO_GATHER_FEW_OBS = 0, 1, 2, 3
_i64p = C.POINTER(C.c_int64)


class VioMapView(C.Structure):
    _fields_ = [
        ("num_frames", C.c_int32), ("num_mappoints", C.c_int32),
        ("frame_Twb", _f32p), ("frame_Tcb", _f32p),
        ("feat_begin", _i32p), ("feat_uv", _f32p), ("feat_valid", _u8p), ("feat_mp", _i32p),
        ("mp_key", _i64p), ("mp_bad", _u8p), ("mp_marg", _u8p), ("mp_pos", _f32p),
        ("mp_obs_begin", _i32p), ("mp_obs_frame", _i32p), ("mp_obs_feat", _i32p),
        ("width", C.c_int32), ("height", C.c_int32), ("boundary_margin", C.c_int32), ("_pad", C.c_int32),
    ]


class VioBaGatherOut(C.Structure):
    _fields_ = [
        ("status", C.c_int32), ("num_lm", C.c_int32), ("num_obs", C.c_int32),
        ("cap_lm", C.c_int32), ("cap_obs", C.c_int32), ("_pad", C.c_int32),
        ("lm_mp", _i32p), ("lm_const", _u8p), ("lm_marg", _u8p), ("lm_xyz", _f64p),
        ("obs_kf", _i32p), ("obs_lm", _i32p), ("obs_uv", _f32p), ("obs_feat", _i32p),
        ("kf_const", _u8p), ("kf_in_problem", _u8p),
        ("T_wb_init", C.POINTER(VioPose)), ("T_cb", C.POINTER(VioPose)),
    ]


class VioBaMapUpdate(C.Structure):
    _fields_ = [
        ("frame_Twb", _f32p), ("frame_set", _u8p), ("frame_vel", _f32p), ("bias", _f32p),
        ("mp_pos", _f32p), ("mp_set", _u8p), ("mp_set_bad", _u8p),
        ("success", C.c_int32), ("num_inliers", C.c_int32), ("num_outliers", C.c_int32),
        ("num_poses_optimized", C.c_int32), ("num_points_optimized", C.c_int32), ("num_iterations", C.c_int32),
        ("initial_cost", C.c_double), ("final_cost", C.c_double),
    ]


class MapView:
    """Owns the numpy arrays of a flat graph (dict with the vio_map_view fields; frame_Twb /
    frame_Tcb (F,4,4) float32, feat_begin (F+1,), feat_uv (G,2), feat_valid / feat_mp (G,), mp_key /
    mp_bad / mp_marg (M,), mp_pos (M,3), optionally mp_obs_begin (M+1,) / mp_obs_frame / mp_obs_feat,
    width, height, boundary_margin) and the vio_map_view pointing at them."""

    def __init__(self, g):
        self.F = int(len(g["feat_begin"]) - 1)
        self.M = int(len(g["mp_key"]))
        self.frame_Twb = np.ascontiguousarray(g["frame_Twb"], np.float32).reshape(-1)
        self.frame_Tcb = np.ascontiguousarray(g["frame_Tcb"], np.float32).reshape(-1)
        self.feat_begin = np.ascontiguousarray(g["feat_begin"], np.int32)
        self.feat_uv = np.ascontiguousarray(g["feat_uv"], np.float32).reshape(-1)
        self.feat_valid = np.ascontiguousarray(g["feat_valid"], np.uint8)
        self.feat_mp = np.ascontiguousarray(g["feat_mp"], np.int32)
        self.mp_key = np.ascontiguousarray(g["mp_key"], np.int64)
        self.mp_bad = np.ascontiguousarray(g["mp_bad"], np.uint8)
        self.mp_marg = np.ascontiguousarray(g["mp_marg"], np.uint8)
        self.mp_pos = np.ascontiguousarray(g["mp_pos"], np.float32).reshape(-1)
        has_obs = g.get("mp_obs_begin") is not None
        self.mp_obs_begin = np.ascontiguousarray(g["mp_obs_begin"], np.int32) if has_obs else None
        self.mp_obs_frame = np.ascontiguousarray(g["mp_obs_frame"], np.int32) if has_obs else None
        self.mp_obs_feat = np.ascontiguousarray(g["mp_obs_feat"], np.int32) if has_obs else None
        v = VioMapView()
        v.num_frames, v.num_mappoints = self.F, self.M
        v.frame_Twb, v.frame_Tcb = _ptr(self.frame_Twb, C.c_float), _ptr(self.frame_Tcb, C.c_float)
        v.feat_begin, v.feat_uv = _ptr(self.feat_begin, C.c_int32), _ptr(self.feat_uv, C.c_float)
        v.feat_valid, v.feat_mp = _ptr(self.feat_valid, C.c_uint8), _ptr(self.feat_mp, C.c_int32)
        v.mp_key, v.mp_bad = _ptr(self.mp_key, C.c_int64), _ptr(self.mp_bad, C.c_uint8)
        v.mp_marg, v.mp_pos = _ptr(self.mp_marg, C.c_uint8), _ptr(self.mp_pos, C.c_float)
        v.mp_obs_begin = _ptr(self.mp_obs_begin, C.c_int32)
        v.mp_obs_frame = _ptr(self.mp_obs_frame, C.c_int32)
        v.mp_obs_feat = _ptr(self.mp_obs_feat, C.c_int32)
        v.width, v.height, v.boundary_margin = int(g["width"]), int(g["height"]), int(g.get("boundary_margin", 20))
        self.c = v

    def obs_capacity(self, variant):
        if variant == VIO_BA_LOCAL:
            return int(self.mp_obs_begin[-1]) if self.mp_obs_begin is not None else 0
        return int(self.feat_begin[-1])


class GatherOut:
    """Caller-owned buffers of one vio_ba_gather call."""

    def __init__(self, view, variant):
        F, M = view.F, view.M
        cap_lm = M if variant != VIO_PNP else int(view.feat_begin[-1])
        cap_obs = view.obs_capacity(variant)
        self.lm_mp = np.zeros(max(cap_lm, 1), np.int32)
        self.lm_const = np.zeros(max(cap_lm, 1), np.uint8)
        self.lm_marg = np.zeros(max(cap_lm, 1), np.uint8)
        self.lm_xyz = np.zeros(3 * max(cap_lm, 1))
        self.obs_kf = np.zeros(max(cap_obs, 1), np.int32)
        self.obs_lm = np.zeros(max(cap_obs, 1), np.int32)
        self.obs_uv = np.zeros(2 * max(cap_obs, 1), np.float32)
        self.obs_feat = np.zeros(max(cap_obs, 1), np.int32)
        self.kf_const = np.zeros(max(F, 1), np.uint8)
        self.kf_in_problem = np.zeros(max(F, 1), np.uint8)
        self.T_wb_init = (VioPose * max(F, 1))()
        self.T_cb = (VioPose * max(F, 1))()
        o = VioBaGatherOut()
        o.cap_lm, o.cap_obs = cap_lm, cap_obs
        o.lm_mp, o.lm_const = _ptr(self.lm_mp, C.c_int32), _ptr(self.lm_const, C.c_uint8)
        o.lm_marg, o.lm_xyz = _ptr(self.lm_marg, C.c_uint8), _ptr(self.lm_xyz, C.c_double)
        o.obs_kf, o.obs_lm = _ptr(self.obs_kf, C.c_int32), _ptr(self.obs_lm, C.c_int32)
        o.obs_uv, o.obs_feat = _ptr(self.obs_uv, C.c_float), _ptr(self.obs_feat, C.c_int32)
        o.kf_const, o.kf_in_problem = _ptr(self.kf_const, C.c_uint8), _ptr(self.kf_in_problem, C.c_uint8)
        o.T_wb_init = C.cast(self.T_wb_init, C.POINTER(VioPose))
        o.T_cb = C.cast(self.T_cb, C.POINTER(VioPose))
        self.F = F
        self.c = o

    def result(self):
        o = self.c
        L, N = o.num_lm, o.num_obs
        return {"status": o.status, "lm_mp": self.lm_mp[:L].copy(), "lm_const": self.lm_const[:L].copy(),
                "lm_marg": self.lm_marg[:L].copy(), "lm_xyz": self.lm_xyz[:3 * L].reshape(-1, 3).copy(),
                "obs_kf": self.obs_kf[:N].copy(), "obs_lm": self.obs_lm[:N].copy(),
                "obs_uv": self.obs_uv[:2 * N].reshape(-1, 2).copy(), "obs_feat": self.obs_feat[:N].copy(),
                "kf_const": self.kf_const[:self.F].copy(), "kf_in_problem": self.kf_in_problem[:self.F].copy(),
                "T_wb_init": poses_from_c(self.T_wb_init, self.F), "T_cb": poses_from_c(self.T_cb, self.F)}

    def window(self, view):
        """The gathered problem as a BaProblem window dict (cols / rows from the view)."""
        r = self.result()
        return {"T_wb_init": r["T_wb_init"], "T_cb": r["T_cb"], "kf_const": r["kf_const"],
                "lm_const": r["lm_const"], "lm_marg": r["lm_marg"], "lm_xyz": r["lm_xyz"],
                "obs_kf": r["obs_kf"], "obs_lm": r["obs_lm"], "obs_uv": r["obs_uv"],
                "cols": float(view.c.width), "rows": float(view.c.height)}


class MapUpdate:
    def __init__(self, view):
        F, M = view.F, view.M
        self.frame_Twb = np.zeros(16 * max(F, 1), np.float32)
        self.frame_set = np.zeros(max(F, 1), np.uint8)
        self.frame_vel = np.zeros(3 * max(F, 1), np.float32)
        self.bias = np.zeros(6, np.float32)
        self.mp_pos = np.zeros(3 * max(M, 1), np.float32)
        self.mp_set = np.zeros(max(M, 1), np.uint8)
        self.mp_set_bad = np.zeros(max(M, 1), np.uint8)
        u = VioBaMapUpdate()
        u.frame_Twb, u.frame_set = _ptr(self.frame_Twb, C.c_float), _ptr(self.frame_set, C.c_uint8)
        u.frame_vel, u.bias = _ptr(self.frame_vel, C.c_float), _ptr(self.bias, C.c_float)
        u.mp_pos, u.mp_set = _ptr(self.mp_pos, C.c_float), _ptr(self.mp_set, C.c_uint8)
        u.mp_set_bad = _ptr(self.mp_set_bad, C.c_uint8)
        self.F, self.M = F, M
        self.c = u

    def result(self):
        u = self.c
        F, M = self.F, self.M
        return {"frame_Twb": self.frame_Twb[:16 * F].reshape(-1, 4, 4).copy(), "frame_set": self.frame_set[:F].copy(),
                "frame_vel": self.frame_vel[:3 * F].reshape(-1, 3).copy(), "bias": self.bias.copy(),
                "mp_pos": self.mp_pos[:3 * M].reshape(-1, 3).copy(), "mp_set": self.mp_set[:M].copy(),
                "mp_set_bad": self.mp_set_bad[:M].copy(),
                "success": u.success, "num_inliers": u.num_inliers, "num_outliers": u.num_outliers,
                "num_poses_optimized": u.num_poses_optimized, "num_points_optimized": u.num_points_optimized,
                "num_iterations": u.num_iterations, "initial_cost": u.initial_cost, "final_cost": u.final_cost}


# ---------------------------------------------------------------------------------------------
# IMU initialisation (vio_imu_init_solve; Optimizer::OptimizeIMUInit)
VIO_IMU_INIT_OK, VIO_IMU_INIT_FEW_FRAMES, VIO_IMU_INIT_NO_PREINT, VIO_IMU_INIT_NO_FACTORS = 0, 1, 2, 3


class VioImuInitProblem(C.Structure):
    _fields_ = [
        ("num_frames", C.c_int32), ("max_iterations", C.c_int32),
        ("T_wb", C.POINTER(VioPose)), ("preint", C.POINTER(VioPreint)), ("preint_valid", _u8p),
        ("gravity_magnitude", C.c_double), ("huber_delta", C.c_double), ("bias_prior_weight", C.c_double),
    ]


class VioImuInitResult(C.Structure):
    _fields_ = [
        ("success", C.c_int32), ("status", C.c_int32), ("iterations", C.c_int32 * 2), ("termination", C.c_int32 * 2),
        ("gravity", C.c_double * 3), ("Rwg", C.c_double * 9), ("gravity_dir", C.c_double * 2), ("scale", C.c_double),
        ("gyro_bias", C.c_double * 3), ("accel_bias", C.c_double * 3), ("initial_cost", C.c_double),
        ("final_cost", C.c_double), ("velocities", _f64p),
    ]


class ImuInitProblem:
    """frames: dict with T_wb (F,4,4) and preint (list of F, entry 0 None / ignored; an entry None for
    a frame without preintegration)."""

    def __init__(self, frames, max_iterations=50, gravity_magnitude=9.81, huber_delta=4.0, bias_prior_weight=1.0):
        self.F = int(len(frames["T_wb"]))
        self.T_wb = poses_to_c(frames["T_wb"])
        pre = list(frames["preint"])
        self.preint, self.valid = preints_to_c([None] + pre[1:] if self.F else [])
        p = VioImuInitProblem()
        p.num_frames = self.F
        p.max_iterations = max_iterations
        p.T_wb = C.cast(self.T_wb, C.POINTER(VioPose))
        p.preint = C.cast(self.preint, C.POINTER(VioPreint))
        p.preint_valid = _ptr(self.valid, C.c_uint8)
        p.gravity_magnitude, p.huber_delta, p.bias_prior_weight = gravity_magnitude, huber_delta, bias_prior_weight
        self.c = p


class ImuInitResult:
    def __init__(self, F):
        self.F = F
        self.vel = np.zeros(3 * max(F, 1))
        r = VioImuInitResult()
        r.velocities = _ptr(self.vel, C.c_double)
        self.c = r

    def result(self):
        r = self.c
        return {"success": r.success, "status": r.status, "iterations": list(r.iterations),
                "termination": list(r.termination), "gravity": np.array(r.gravity[:]),
                "Rwg": np.array(r.Rwg[:]).reshape(3, 3), "gravity_dir": np.array(r.gravity_dir[:]),
                "scale": r.scale, "gyro_bias": np.array(r.gyro_bias[:]), "accel_bias": np.array(r.accel_bias[:]),
                "initial_cost": r.initial_cost, "final_cost": r.final_cost,
                "velocities": self.vel[: 3 * self.F].reshape(-1, 3).copy()}


# ---------------------------------------------------------------------------------------------
# Monocular initialisation (vio_mono_init_solve; Initializer::TryMonocularInitialization)
VIO_INIT_OK, VIO_INIT_TOO_FEW_BEARINGS, VIO_INIT_ESSENTIAL_FAILED, VIO_INIT_POSE_FAILED = 0, 1, 2, 3
VIO_INIT_TRIANGULATION, VIO_INIT_VALIDATION = 4, 5


class VioMonoInitParams(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32), ("min_features", C.c_int32), ("ransac_iterations", C.c_int32),
        ("ransac_threshold", C.c_float), ("max_reprojection_error", C.c_float),
    ]


class VioMonoInitResult(C.Structure):
    _fields_ = [
        ("status", C.c_int32), ("best_hypothesis", C.c_int32), ("num_inliers", C.c_int32),
        ("pose_candidate", C.c_int32), ("candidate_good", C.c_int32 * 4), ("num_triangulated", C.c_int32),
        ("num_valid", C.c_int32), ("mean_reproj_error", C.c_float), ("scale_factor", C.c_float),
        ("E", C.c_float * 9), ("R", C.c_float * 9), ("t", C.c_float * 3),
    ]


def mono_init_params(width=960, height=480, min_features=100, ransac_iterations=200, ransac_threshold=0.1,
                     max_reprojection_error=5.0):
    """Defaults: config/default_config.yaml:33-41 (initialization.*) at the demo's 960x480."""
    p = VioMonoInitParams()
    p.width, p.height, p.min_features, p.ransac_iterations = width, height, min_features, ransac_iterations
    p.ransac_threshold, p.max_reprojection_error = ransac_threshold, max_reprojection_error
    return p


def mono_init_result_dict(r):
    return {
        "status": r.status, "best_hypothesis": r.best_hypothesis, "num_inliers": r.num_inliers,
        "pose_candidate": r.pose_candidate, "candidate_good": list(r.candidate_good),
        "num_triangulated": r.num_triangulated, "num_valid": r.num_valid,
        "mean_reproj_error": r.mean_reproj_error, "scale_factor": r.scale_factor,
        "E": np.array(r.E, np.float32).reshape(3, 3), "R": np.array(r.R, np.float32).reshape(3, 3),
        "t": np.array(r.t, np.float32),
    }


# ---------------------------------------------------------------------------------------------
# Estimator window bookkeeping (vio_window_*; Estimator::CreateKeyframe / TriangulateNewMapPoints)
_i32p = C.POINTER(C.c_int32)
_f32p = C.POINTER(C.c_float)


class VioWindowFrame(C.Structure):
    _fields_ = [
        ("frame_id", C.c_int32), ("num_features", C.c_int32), ("width", C.c_int32), ("_pad", C.c_int32),
        ("T_wb", _f32p), ("T_bc", _f32p), ("feature_id", _i32p), ("uv", _f32p), ("bearing", _f32p),
        ("valid", _u8p), ("mappoint", _i32p), ("track_begin", _i32p), ("track_frame", _i32p), ("track_feat", _i32p),
    ]


class VioWindowKfStats(C.Structure):
    _fields_ = [("obs_added", C.c_int32), ("transferred", C.c_int32), ("deleted", C.c_int32),
                ("removed_frame", C.c_int32), ("num_keyframes", C.c_int32), ("_pad", C.c_int32)]


class VioWindowMappointInfo(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("bad", C.c_int32), ("marginalized", C.c_int32), ("triangulated", C.c_int32),
                ("reference_frame", C.c_int32), ("num_observations", C.c_int32)]
