"""MI355X-native hot path of 93won/360_visual_inertial_odometry: ERP feature tracking + sliding-window BA.

The compute path is libvio360.so (HIP kernels for gfx950 behind the C-ABI in include/vio360.h).
This module only loads it and marshals numpy buffers; there is no CPU fallback: if the library or
a GPU is missing every entry point raises.
"""
import ctypes as C
import os
import weakref

import numpy as np

from . import abi
from .abi import (VIO_BA_FULL, VIO_BA_LOCAL, VIO_BA_VI, VIO_PNP, BaOutput, BaProblem,  # noqa: F401
                  ErpFrontendParams, ErpKltParams, ErpTrackerParams, default_frontend_params,
                  default_klt_params, default_tracker_params)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VIO360_LIB") or os.path.join(_HERE, "libvio360.so")
_lib = None

EXPORTS = [
    "vio_abi_version", "vio_ctx_create", "vio_ctx_destroy", "vio_ctx_last_error",
    "vio_ba_solve", "vio_ba_solve_batched", "vio_ba_batch_create", "vio_ba_batch_run",
    "vio_ba_batch_sync", "vio_ba_batch_download", "vio_ba_batch_kernel_ms", "vio_ba_batch_destroy",
    "vio_ba_batch_route",
    "vio_ba_batch_profile", "vio_ba_batch_phase_cycles",
    "erp_klt_track", "erp_gftt", "erp_rot_ransac", "erp_ransac_samples", "erp_tracker_create",
    "erp_tracker_upload", "erp_tracker_device_frame", "erp_tracker_swap", "erp_tracker_set_points",
    "erp_tracker_run", "erp_tracker_sync", "erp_tracker_download", "erp_tracker_stage_ms",
    "erp_tracker_gftt_fallbacks",
    "erp_tracker_set_stage_timing",
    "erp_tracker_destroy", "erp_frontend_create", "erp_frontend_track", "erp_frontend_features",
    "erp_frontend_stats", "erp_frontend_destroy", "vio_imu_preintegrate", "vio_imu_preintegrate_kernel_ms", "vio_imu_preintegrate_device",
    "vio_ba_batch_set_preint",
    "vio_triangulate", "vio_triangulate_device", "vio_triangulate_kernel_ms",
    "vio_load_camera_timestamps", "vio_load_imu_csv", "erp_resize_area", "erp_resize_area_device",
    "erp_resize_area_kernel_ms", "erp_tracker_upload_resized",
    "vio_ba_record_bytes", "vio_ba_batch_record_bytes", "vio_ba_batch_pack", "vio_ba_record_unpack",
    "vio_ba_gather", "vio_ba_write_back", "vio_imu_init_solve",
    "vio_mono_init_solve", "vio_mono_init_kernel_ms", "vio_mono_init_samples", "vio_init_select_features",
    "vio_init_parallax", "vio_init_compose", "vio_ctx_set_ba_route",
    "vio_window_create", "vio_window_destroy", "vio_window_add_mappoint", "vio_window_add_observation",
    "vio_window_link_mappoints", "vio_window_add_keyframe", "vio_window_triangulation_candidates",
    "vio_window_commit_triangulation", "vio_window_triangulate", "vio_window_keyframes", "vio_window_num_mappoints",
    "vio_window_mappoint", "vio_window_mappoint_observations", "vio_window_frame_mappoints", "vio_window_map_view",
    "vio_window_apply_update", "vio_lie_eval",
]


class VioError(RuntimeError):
    pass


def lib():
    """Load libvio360.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise VioError(f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback exists)")
    L = C.CDLL(LIB_PATH)
    L.vio_ctx_last_error.restype = C.c_char_p
    L.vio_ctx_last_error.argtypes = [C.c_void_p]
    L.vio_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.vio_ctx_destroy.argtypes = [C.c_void_p]
    L.vio_ba_solve_batched.argtypes = [C.c_void_p, C.POINTER(abi.VioBaProblem), C.POINTER(abi.VioBaOutput), C.c_int]
    L.vio_ba_batch_create.argtypes = [C.c_void_p, C.POINTER(abi.VioBaProblem), C.c_int, C.POINTER(C.c_void_p)]
    L.vio_ba_batch_run.argtypes = [C.c_void_p]
    L.vio_ba_batch_sync.argtypes = [C.c_void_p]
    L.vio_ba_batch_download.argtypes = [C.c_void_p, C.POINTER(abi.VioBaOutput)]
    L.vio_ba_batch_kernel_ms.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int)]
    if hasattr(L, "vio_ba_batch_route") or "VIO360_LIB" not in os.environ:  # (A/B runs may load older builds)
        L.vio_ba_batch_route.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.vio_ba_batch_destroy.argtypes = [C.c_void_p]
    L.vio_ba_batch_profile.argtypes = [C.c_void_p, C.c_int]
    L.vio_ba_batch_phase_cycles.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    vp = C.c_void_p
    L.erp_klt_track.argtypes = [vp, vp, vp, C.c_int, C.c_int, C.c_int, vp, C.c_int, vp, vp, vp,
                                C.POINTER(abi.ErpKltParams)]
    L.erp_gftt.argtypes = [vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, vp,
                           C.POINTER(C.c_int)]
    L.erp_rot_ransac.argtypes = [vp, vp, vp, C.c_int, C.c_int, C.c_int, vp, C.c_int, C.c_float, vp,
                                 C.POINTER(C.c_int)]
    L.erp_ransac_samples.argtypes = [C.c_uint32, C.c_int, C.c_int, vp]
    L.erp_tracker_create.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.erp_tracker_upload.argtypes = [vp, C.c_int, vp, C.c_int]
    L.erp_tracker_device_frame.argtypes = [vp, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_int)]
    L.erp_tracker_swap.argtypes = [vp]
    L.erp_tracker_set_points.argtypes = [vp, vp, C.c_int]
    L.erp_tracker_run.argtypes = [vp, C.POINTER(abi.ErpKltParams), C.POINTER(abi.ErpTrackerParams)]
    L.erp_tracker_sync.argtypes = [vp]
    L.erp_tracker_download.argtypes = [vp, vp, vp, vp, vp, C.POINTER(C.c_int)]
    L.erp_tracker_stage_ms.argtypes = [vp] + [C.POINTER(C.c_double)] * 5
    if hasattr(L, "erp_tracker_gftt_fallbacks") or "VIO360_LIB" not in os.environ:  # (A/B: older builds)
        L.erp_tracker_gftt_fallbacks.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.erp_tracker_set_stage_timing.argtypes = [vp, C.c_int]
    L.erp_tracker_destroy.argtypes = [vp]
    L.erp_frontend_create.argtypes = [vp, C.c_int, C.c_int, C.POINTER(abi.ErpFrontendParams), C.POINTER(C.c_void_p)]
    L.erp_frontend_track.argtypes = [vp, vp, C.c_int, C.POINTER(C.c_int)]
    L.erp_frontend_features.argtypes = [vp, vp, vp, vp, vp, C.c_int]
    L.erp_frontend_stats.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.erp_frontend_destroy.argtypes = [vp]
    L.vio_imu_preintegrate.argtypes = [vp, vp, C.c_int, vp, vp, C.c_int, vp, vp, C.POINTER(abi.VioImuNoise), vp,
                                       vp, vp]
    L.vio_imu_preintegrate_kernel_ms.argtypes = [vp, C.POINTER(C.c_double)]
    L.vio_imu_preintegrate_device.argtypes = [vp, vp, C.c_int, vp, vp, C.c_int, vp, vp, C.POINTER(abi.VioImuNoise),
                                              vp, vp, vp]
    L.vio_ba_batch_set_preint.argtypes = [vp, vp, C.c_int, C.c_int]
    L.vio_triangulate.argtypes = [vp, vp, C.c_int, vp, vp, C.c_int, C.c_int, vp, vp, vp]
    L.vio_triangulate_device.argtypes = [vp, vp, C.c_int, vp, vp, C.c_int, C.c_int, vp, vp, vp]
    L.vio_triangulate_kernel_ms.argtypes = [vp, C.POINTER(C.c_double)]
    L.vio_lie_eval.argtypes = [vp, C.c_int, vp, C.c_int, vp]
    L.vio_load_camera_timestamps.argtypes = [C.c_char_p, vp, C.c_int, C.POINTER(C.c_int)]
    L.vio_load_imu_csv.argtypes = [C.c_char_p, vp, C.c_int, C.POINTER(C.c_int)]
    L.erp_resize_area.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, vp, C.c_int, C.c_int, C.c_int]
    L.erp_resize_area_device.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_int, C.c_int, C.c_int]
    L.erp_resize_area_kernel_ms.argtypes = [vp, C.POINTER(C.c_double)]
    L.erp_tracker_upload_resized.argtypes = [vp, C.c_int, vp, C.c_int, C.c_int, C.c_int]
    L.vio_ba_record_bytes.argtypes = [C.c_int, C.c_int, C.c_int]
    L.vio_ba_record_bytes.restype = C.c_size_t
    L.vio_ba_batch_record_bytes.argtypes = [vp, C.POINTER(C.c_size_t)]
    L.vio_ba_batch_pack.argtypes = [vp, vp, C.c_int]
    L.vio_ba_record_unpack.argtypes = [vp, C.c_size_t, C.POINTER(abi.VioBaOutput)]
    L.vio_ba_gather.argtypes = [C.POINTER(abi.VioMapView), C.c_int, C.c_int, C.c_int, C.POINTER(abi.VioBaGatherOut)]
    L.vio_ba_write_back.argtypes = [C.POINTER(abi.VioMapView), C.c_int, C.POINTER(abi.VioBaGatherOut),
                                    C.POINTER(abi.VioBaOutput), C.POINTER(abi.VioBaMapUpdate)]
    L.vio_imu_init_solve.argtypes = [vp, C.POINTER(abi.VioImuInitProblem), C.POINTER(abi.VioImuInitResult), C.c_int]
    L.vio_mono_init_solve.argtypes = [vp, vp, vp, C.c_int, vp, C.POINTER(abi.VioMonoInitParams),
                                      C.POINTER(abi.VioMonoInitResult), vp, vp]
    L.vio_mono_init_kernel_ms.argtypes = [vp, C.POINTER(C.c_double)]
    L.vio_mono_init_samples.argtypes = [C.c_uint32, C.c_int, C.c_int, vp]
    L.vio_init_select_features.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                           vp, C.POINTER(C.c_int)]
    L.vio_init_parallax.argtypes = [vp, vp, C.c_int, vp, vp, C.c_int, C.POINTER(C.c_float)]
    L.vio_init_compose.argtypes = [vp, vp, vp, vp, vp, vp, C.c_int]
    L.vio_ctx_set_ba_route.argtypes = [vp, C.c_int]
    L.vio_window_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.vio_window_destroy.argtypes = [vp]
    L.vio_window_add_mappoint.argtypes = [vp, vp, C.c_int32, C.POINTER(C.c_int32)]
    L.vio_window_add_observation.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32]
    L.vio_window_link_mappoints.argtypes = [vp, vp, vp, vp, C.c_int, vp, C.c_int, vp]
    L.vio_window_add_keyframe.argtypes = [vp, C.POINTER(abi.VioWindowFrame), C.POINTER(abi.VioWindowKfStats)]
    L.vio_window_triangulation_candidates.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp, C.c_int,
                                                      C.POINTER(C.c_int)]
    L.vio_window_commit_triangulation.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp, C.c_int, vp,
                                                  C.POINTER(C.c_int)]
    L.vio_window_triangulate.argtypes = [vp, vp, C.c_int32, C.c_int32, C.POINTER(C.c_int)]
    L.vio_window_keyframes.argtypes = [vp, vp, C.c_int, C.POINTER(C.c_int)]
    L.vio_window_num_mappoints.argtypes = [vp]
    L.vio_window_mappoint.argtypes = [vp, C.c_int32, C.POINTER(abi.VioWindowMappointInfo)]
    L.vio_window_mappoint_observations.argtypes = [vp, C.c_int32, vp, vp, C.c_int, C.POINTER(C.c_int)]
    L.vio_window_frame_mappoints.argtypes = [vp, C.c_int32, vp, C.c_int, C.POINTER(C.c_int)]
    L.vio_window_map_view.argtypes = [vp, C.c_int, C.c_int, C.POINTER(abi.VioMapView)]
    L.vio_window_apply_update.argtypes = [vp, C.POINTER(abi.VioBaMapUpdate)]
    _lib = L
    return L


class Context:
    """vio_ctx wrapper: one HIP device + stream."""

    def __init__(self, device=0):
        L = lib()
        h = C.c_void_p()
        rc = L.vio_ctx_create(int(device), C.byref(h))
        if rc != 0:
            raise VioError(f"vio_ctx_create failed ({rc}): {L.vio_ctx_last_error(None).decode()}")
        self.h = h
        self._children = weakref.WeakSet()  # batches / trackers: closed before the context

    def check(self, rc, what):
        if rc != 0:
            raise VioError(f"{what} failed ({rc}): {lib().vio_ctx_last_error(self.h).decode()}")

    def close(self):
        if self.h:
            for ch in list(self._children):  # the C-ABI requires children to go first
                try:
                    ch.close()
                except Exception:
                    pass
            lib().vio_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- bundle adjustment ----
    ROUTE_AUTO, ROUTE_PHASES, ROUTE_SINGLE_KERNEL, ROUTE_CLUSTER = 0, 1, 2, 3

    def set_ba_route(self, route):
        """vio_ctx_set_ba_route: execution route of later window solves on this context."""
        self.check(lib().vio_ctx_set_ba_route(self.h, int(route)), "vio_ctx_set_ba_route")

    LIE_SO3_EXP, LIE_SE3_EXP, LIE_IMU_LOG, LIE_SO3D_EXP, LIE_SO3D_LOG = range(5)
    _LIE_IO = {0: (3, 9), 1: (6, 12), 2: (9, 3), 3: (3, 9), 4: (9, 3)}

    def lie_eval(self, op, x):
        """vio_lie_eval: the device Lie maths of the BA factors (LIE_* ops) over the rows of x."""
        ni, no = self._LIE_IO[int(op)]
        a = np.ascontiguousarray(np.asarray(x, np.float64).reshape(-1, ni))
        out = np.zeros((max(len(a), 1), no), np.float64)
        self.check(lib().vio_lie_eval(self.h, int(op), _p(a), len(a), _p(out)), "vio_lie_eval")
        return out[:len(a)]

    def ba_solve(self, problems):
        """Solve a list of BaProblem windows in one launch; returns list of result dicts."""
        n = len(problems)
        P = (abi.VioBaProblem * n)(*[p.c for p in problems])
        outs = [BaOutput(p.K, p.L, p.N) for p in problems]
        O = (abi.VioBaOutput * n)(*[o.c for o in outs])
        self.check(lib().vio_ba_solve_batched(self.h, P, O, n), "vio_ba_solve_batched")
        return [o.result() for o in outs]

    def ba_solve_call(self, problems, trace_cap=256):
        """vio_ba_solve_batched with its problem / output structs marshalled once: call() is one C-ABI call
        (pack + upload + solve + download, as a C++ host makes it per keyframe), results() converts the
        outputs of the last call."""
        return BaSolveCall(self, problems, trace_cap)

    # ---- IMU initialisation ----
    def imu_init(self, problems):
        """vio_imu_init_solve: Optimizer::OptimizeIMUInit for a list of abi.ImuInitProblem in one
        launch (one workgroup each); returns the result dicts."""
        n = len(problems)
        P = (abi.VioImuInitProblem * max(n, 1))(*[p.c for p in problems])
        outs = [abi.ImuInitResult(p.F) for p in problems]
        R = (abi.VioImuInitResult * max(n, 1))(*[o.c for o in outs])
        self.check(lib().vio_imu_init_solve(self.h, P, R, n), "vio_imu_init_solve")
        for k, o in enumerate(outs):
            o.c = R[k]
        return [o.result() for o in outs]


    # ---- monocular initialisation ----
    def mono_init(self, bearings1, bearings2, samples, params=None):
        """vio_mono_init_solve: Initializer::TryMonocularInitialization's numeric core on device.
        bearings1/2 (n,3) f32 unit bearings, samples (iters,8) int32 (mono_init_samples).  Returns
        (result dict, inlier mask (n,) u8, points (n,3) f32 in camera-1 coordinates, scaled)."""
        b1 = np.ascontiguousarray(bearings1, np.float32).reshape(-1, 3)
        b2 = np.ascontiguousarray(bearings2, np.float32).reshape(-1, 3)
        n = len(b1)
        S = np.ascontiguousarray(samples, np.int32).reshape(-1, 8)
        P = params if params is not None else abi.mono_init_params(ransac_iterations=len(S))
        R = abi.VioMonoInitResult()
        M = np.zeros(max(n, 1), np.uint8)
        X = np.zeros((max(n, 1), 3), np.float32)
        self.check(lib().vio_mono_init_solve(self.h, _p(b1), _p(b2), n, _p(S), C.byref(P), C.byref(R), _p(M), _p(X)),
                   "vio_mono_init_solve")
        return abi.mono_init_result_dict(R), M[:n], X[:n]

    def mono_init_kernel_ms(self):
        ms = C.c_double()
        self.check(lib().vio_mono_init_kernel_ms(self.h, C.byref(ms)), "vio_mono_init_kernel_ms")
        return ms.value

    # ---- IMU preintegration ----
    def imu_preintegrate(self, samples, t_start, t_end, gyro_bias=None, accel_bias=None, noise=None):
        """IMUPreintegrator::Preintegrate for every interval [t_start[i], t_end[i]) in one launch.

        samples: (M, 7) [t, ax, ay, az, gx, gy, gz] rows sorted by t (or vio_imu_data records).
        Returns (records dict of (n, ...) arrays, valid (n,) u8, cov_bias_diag (n, 6) f32)."""
        return _imu_call(lambda *a: lib().vio_imu_preintegrate(self.h, *a), self.check, samples, t_start, t_end,
                         gyro_bias, accel_bias, noise)

    def imu_preintegrate_device(self, imu_ptr, n_imu, t0_ptr, t1_ptr, n, out_ptr, valid_ptr, cov_bias_ptr,
                                gyro_bias_ptr=None, accel_bias_ptr=None, noise=None):
        """vio_imu_preintegrate_device on raw device pointers (ints), async on the context stream."""
        nz = abi.imu_noise(noise)
        self.check(lib().vio_imu_preintegrate_device(self.h, imu_ptr, n_imu, t0_ptr, t1_ptr, n, gyro_bias_ptr,
                                                     accel_bias_ptr, C.byref(nz), out_ptr, valid_ptr, cov_bias_ptr),
                   "vio_imu_preintegrate_device")

    def imu_kernel_ms(self):
        ms = C.c_double()
        self.check(lib().vio_imu_preintegrate_kernel_ms(self.h, C.byref(ms)), "vio_imu_preintegrate_kernel_ms")
        return ms.value

    # ---- two-view triangulation ----
    def triangulate(self, T_cw, pairs, bearings, width):
        """Estimator::TriangulateSinglePoint for n candidates: T_cw (m,4,4) world-to-camera f32,
        pairs (n,2) pose indices, bearings (n,6) = (b1, b2).  Returns (points (n,3) f32,
        valid (n,) u8, pixel_err (n,2) f32)."""
        T = np.ascontiguousarray(T_cw, dtype=np.float32).reshape(-1, 16)
        P = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1, 2)
        B = np.ascontiguousarray(bearings, dtype=np.float32).reshape(-1, 6)
        if len(P) != len(B):
            raise ValueError("pairs / bearings sizes differ")
        n = len(P)
        X = np.zeros((max(n, 1), 3), np.float32)
        V = np.zeros(max(n, 1), np.uint8)
        E = np.zeros((max(n, 1), 2), np.float32)
        self.check(lib().vio_triangulate(self.h, _p(T), len(T), _p(P), _p(B), n, int(width), _p(X), _p(V), _p(E)),
                   "vio_triangulate")
        return X[:n], V[:n], E[:n]

    def triangulate_device(self, T_ptr, n_poses, pair_ptr, bear_ptr, n, width, x_ptr, valid_ptr, err_ptr=None):
        """vio_triangulate_device on raw device pointers (ints), async on the context stream."""
        self.check(lib().vio_triangulate_device(self.h, T_ptr, n_poses, pair_ptr, bear_ptr, n, int(width), x_ptr,
                                                valid_ptr, err_ptr), "vio_triangulate_device")

    def triangulate_kernel_ms(self):
        ms = C.c_double()
        self.check(lib().vio_triangulate_kernel_ms(self.h, C.byref(ms)), "vio_triangulate_kernel_ms")
        return ms.value

    # ---- frame preprocessing ----
    def resize_area(self, img, dW, dH):
        """cv::resize(..., INTER_AREA) of a u8 frame to (dW, dH), integer factors (app/main.cpp:203)."""
        a = _u8img(img)
        H, W = a.shape
        out = np.zeros((dH, dW), np.uint8)
        self.check(lib().erp_resize_area(self.h, _p(a), W, H, a.strides[0], _p(out), dW, dH, dW), "erp_resize_area")
        return out

    def resize_area_device(self, src_ptr, W, H, stride, n_frames, dst_ptr, dW, dH, dst_stride):
        self.check(lib().erp_resize_area_device(self.h, src_ptr, W, H, stride, n_frames, dst_ptr, dW, dH, dst_stride),
                   "erp_resize_area_device")

    def resize_kernel_ms(self):
        ms = C.c_double()
        self.check(lib().erp_resize_area_kernel_ms(self.h, C.byref(ms)), "erp_resize_area_kernel_ms")
        return ms.value

    # ---- ERP feature tracking ----
    def klt_track(self, prev, curr, pts, params=None):
        """cv::calcOpticalFlowPyrLK as FeatureTracker::TrackOpticalFlow calls it -> (next, status, err)."""
        prev, curr = _u8img(prev), _u8img(curr)
        H, W = prev.shape
        pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 2)
        n = len(pts)
        nxt = np.zeros((n, 2), np.float32)
        st = np.zeros(n, np.uint8)
        err = np.zeros(n, np.float32)
        prm = params or default_klt_params()
        self.check(lib().erp_klt_track(self.h, _p(prev), _p(curr), W, H, W, _p(pts), n, _p(nxt), _p(st), _p(err),
                                       C.byref(prm)), "erp_klt_track")
        return nxt, st, err

    def gftt(self, img, mask=None, max_corners=1000, quality=0.01, min_dist=30.0):
        """cv::goodFeaturesToTrack(blockSize 3, useHarris false) -> (k, 2) float32 corners."""
        img = _u8img(img)
        H, W = img.shape
        m = None if mask is None else _u8img(mask)
        cap = max_corners if max_corners > 0 else W * H
        out = np.zeros((cap, 2), np.float32)
        n = C.c_int()
        self.check(lib().erp_gftt(self.h, _p(img), _p(m) if m is not None else None, W, H, W, int(max_corners),
                                  float(quality), float(min_dist), _p(out), C.byref(n)), "erp_gftt")
        return out[: n.value].copy()

    def rot_ransac(self, p0, p1, W, H, samples, thresh_rad=None):
        """RejectOutliersRotationRANSAC on an injected sample stream -> (mask u8, n_inliers)."""
        p0 = np.ascontiguousarray(p0, np.float32).reshape(-1, 2)
        p1 = np.ascontiguousarray(p1, np.float32).reshape(-1, 2)
        samples = np.ascontiguousarray(samples, np.int32).reshape(-1)
        n = len(p0)
        thr = ransac_threshold() if thresh_rad is None else thresh_rad
        mask = np.zeros(n, np.uint8)
        nin = C.c_int()
        self.check(lib().erp_rot_ransac(self.h, _p(p0), _p(p1), n, W, H, _p(samples), len(samples) // 3,
                                        float(thr), _p(mask), C.byref(nin)), "erp_rot_ransac")
        return mask, nin.value


def load_camera_timestamps(path):
    """LoadCameraTimestamps (app/main.cpp:30-48) through the C-ABI: (n,) f64."""
    L, n = lib(), C.c_int()
    rc = L.vio_load_camera_timestamps(os.fsencode(path), None, 0, C.byref(n))
    if rc:
        raise VioError(f"vio_load_camera_timestamps({path}) failed ({rc})")
    out = np.zeros(max(n.value, 1), np.float64)
    L.vio_load_camera_timestamps(os.fsencode(path), _p(out), n.value, C.byref(n))
    return out[:n.value]


def load_imu_csv(path):
    """LoadIMUData (app/main.cpp:50-90) through the C-ABI: vio_imu_data records (abi.IMU_DTYPE)."""
    L, n = lib(), C.c_int()
    rc = L.vio_load_imu_csv(os.fsencode(path), None, 0, C.byref(n))
    if rc:
        raise VioError(f"vio_load_imu_csv({path}) failed ({rc})")
    out = np.zeros(max(n.value, 1), abi.IMU_DTYPE)
    L.vio_load_imu_csv(os.fsencode(path), _p(out), n.value, C.byref(n))
    return out[:n.value]


def _imu_call(fn, check, samples, t_start, t_end, gyro_bias, accel_bias, noise):
    """Marshal one vio_imu_preintegrate-shaped call (shared by the HIP path and the test oracle)."""
    imu = samples if getattr(samples, "dtype", None) == abi.IMU_DTYPE else abi.imu_array(samples)
    imu = np.ascontiguousarray(imu)
    t0 = np.ascontiguousarray(t_start, dtype=np.float64).reshape(-1)
    t1 = np.ascontiguousarray(t_end, dtype=np.float64).reshape(-1)
    if t0.shape != t1.shape:
        raise ValueError("t_start / t_end sizes differ")
    n = len(t0)
    bg = None if gyro_bias is None else np.ascontiguousarray(np.broadcast_to(np.asarray(gyro_bias, np.float32), (n, 3)))
    ba = None if accel_bias is None else np.ascontiguousarray(np.broadcast_to(np.asarray(accel_bias, np.float32), (n, 3)))
    out = (abi.VioPreint * max(n, 1))()
    valid = np.zeros(max(n, 1), np.uint8)
    cov_bias = np.zeros((max(n, 1), 6), np.float32)
    nz = abi.imu_noise(noise)
    rc = fn(_p(imu), len(imu), _p(t0), _p(t1), n, None if bg is None else _p(bg), None if ba is None else _p(ba),
            C.byref(nz), C.cast(out, C.c_void_p), _p(valid), _p(cov_bias))
    check(rc, "vio_imu_preintegrate")
    rec = abi.preint_records(out)
    return {k: v[:n] for k, v in rec.items()}, valid[:n], cov_bias[:n]


def record_bytes(K, L, N):
    """vio_ba_record_bytes: size of a packed result record of a K x L x N window."""
    return int(lib().vio_ba_record_bytes(K, L, N))


def unpack_record(rec):
    """vio_ba_record_unpack (host): one packed record (uint8 array) -> result dict (no chi2 / trace)."""
    rec = np.ascontiguousarray(rec, np.uint8)
    if rec.size < 16:
        raise VioError("vio_ba_record_unpack: record shorter than its header")
    K, L, N = (int(v) for v in rec[:12].view(np.int32))
    if K <= 0 or L < 0 or N < 0 or record_bytes(K, L, N) > rec.size:
        raise VioError(f"vio_ba_record_unpack: header K={K} L={L} N={N} does not fit a {rec.size}-byte record")
    o = BaOutput(K, L, N)
    rc = lib().vio_ba_record_unpack(_p(rec), rec.size, C.byref(o.c))
    if rc != 0:
        raise VioError(f"vio_ba_record_unpack failed ({rc})")
    r = o.result()
    del r["obs_chi2"], r["trace"]
    return r


def _u8img(a):
    return np.ascontiguousarray(a, np.uint8)


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def ransac_threshold(deg=2.0):
    """threshold_rad = m_ransac_threshold * M_PI / 180.0f (FeatureTracker.cpp:305), as float."""
    return float(np.float32(np.float64(np.float32(deg)) * np.pi / np.float64(np.float32(180.0))))


def mono_init_samples(seed, n, iters=200):
    """Initializer::ComputeEssentialMatrix's sample stream (8 distinct indices per hypothesis) with an
    injected seed (the reference seeds from std::random_device)."""
    out = np.zeros((max(iters, 1), 8), np.int32)
    rc = lib().vio_mono_init_samples(int(seed) & 0xffffffff, int(n), int(iters), _p(out))
    if rc:
        raise VioError(f"vio_mono_init_samples failed ({rc})")
    return out[:iters]


def init_select_features(uv, obs_count, width, height, grid_cols=20, grid_rows=10, min_observations=10,
                         min_features=100):
    """Initializer::SelectFeaturesForInit on flat arrays; returns the selected feature indices."""
    uv = np.ascontiguousarray(uv, np.float32).reshape(-1, 2)
    oc = np.ascontiguousarray(obs_count, np.int32)
    n = len(uv)
    out = np.zeros(max(n, 1), np.int32)
    m = C.c_int()
    rc = lib().vio_init_select_features(_p(uv), _p(oc), n, width, height, grid_cols, grid_rows, min_observations,
                                        min_features, _p(out), C.byref(m))
    if rc:
        raise VioError(f"vio_init_select_features failed ({rc})")
    return out[:m.value]


def init_parallax(ids1, uv1, ids2, uv2):
    """Initializer::ComputeParallax: median pixel displacement of id-matched features."""
    i1 = np.ascontiguousarray(ids1, np.int32)
    i2 = np.ascontiguousarray(ids2, np.int32)
    u1 = np.ascontiguousarray(uv1, np.float32).reshape(-1, 2)
    u2 = np.ascontiguousarray(uv2, np.float32).reshape(-1, 2)
    out = C.c_float()
    rc = lib().vio_init_parallax(_p(i1), _p(u1), len(i1), _p(i2), _p(u2), len(i2), C.byref(out))
    if rc:
        raise VioError(f"vio_init_parallax failed ({rc})")
    return out.value


def init_compose(T_BC, R, t, points=None):
    """Initializer.cpp:174-224: returns (T_wb1, T_wb2, world points or None)."""
    T = np.ascontiguousarray(T_BC, np.float32).reshape(4, 4)
    Rm = np.ascontiguousarray(R, np.float32).reshape(3, 3)
    tv = np.ascontiguousarray(t, np.float32).reshape(3)
    T1 = np.zeros((4, 4), np.float32)
    T2 = np.zeros((4, 4), np.float32)
    X = None if points is None else np.array(points, np.float32).reshape(-1, 3).copy()
    rc = lib().vio_init_compose(_p(T), _p(Rm), _p(tv), _p(T1), _p(T2), None if X is None else _p(X),
                                0 if X is None else len(X))
    if rc:
        raise VioError(f"vio_init_compose failed ({rc})")
    return T1, T2, X


def ransac_samples(seed, n, iters=1000):
    """The reference's mt19937 + uniform_int_distribution sample stream with an injected seed."""
    out = np.zeros(3 * iters, np.int32)
    rc = lib().erp_ransac_samples(int(seed) & 0xffffffff, int(n), int(iters), _p(out))
    if rc != 0:
        raise VioError(f"erp_ransac_samples failed ({rc})")
    return out


class Tracker:
    """Device-resident frame pipeline (erp_tracker_*): pyramids + LK + RANSAC + GFTT re-detection."""

    def __init__(self, ctx, W, H, max_points=2048, max_corners=2048):
        self.ctx, self.W, self.H = ctx, W, H
        self.max_points, self.max_corners = max_points, max_corners
        h = C.c_void_p()
        ctx.check(lib().erp_tracker_create(ctx.h, W, H, max_points, max_corners, C.byref(h)), "erp_tracker_create")
        self.h = h
        ctx._children.add(self)
        self.n = 0

    def upload(self, slot, img):
        img = _u8img(img)
        self.ctx.check(lib().erp_tracker_upload(self.h, slot, _p(img), img.shape[1]), "erp_tracker_upload")

    def upload_resized(self, slot, img):
        """erp_tracker_upload_resized: a camera-resolution frame, INTER_AREA-resized on the device."""
        img = _u8img(img)
        H, W = img.shape
        self.ctx.check(lib().erp_tracker_upload_resized(self.h, slot, _p(img), W, H, img.strides[0]),
                       "erp_tracker_upload_resized")

    def swap(self):
        self.ctx.check(lib().erp_tracker_swap(self.h), "erp_tracker_swap")

    def set_points(self, pts):
        pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 2)
        self.n = len(pts)
        self._pts = pts
        self.ctx.check(lib().erp_tracker_set_points(self.h, _p(pts), self.n), "erp_tracker_set_points")

    def run(self, params=None, klt=None):
        prm = params or default_tracker_params()
        kp = klt or default_klt_params()
        self.ctx.check(lib().erp_tracker_run(self.h, C.byref(kp), C.byref(prm)), "erp_tracker_run")

    def sync(self):
        self.ctx.check(lib().erp_tracker_sync(self.h), "erp_tracker_sync")

    def download(self):
        n = self.n
        nxt = np.zeros((max(n, 1), 2), np.float32)
        st = np.zeros(max(n, 1), np.uint8)
        kept = np.zeros(max(n, 1), np.uint8)
        cor = np.zeros((self.max_corners, 2), np.float32)
        nc = C.c_int()
        self.ctx.check(lib().erp_tracker_download(self.h, _p(nxt), _p(st), _p(kept), _p(cor), C.byref(nc)),
                       "erp_tracker_download")
        return {"next": nxt[:n], "status": st[:n], "kept": kept[:n], "corners": cor[: nc.value].copy()}

    def set_stage_timing(self, on):
        """Record the per-stage events on the next runs (on) or only the pipeline's start and end."""
        self.ctx.check(lib().erp_tracker_set_stage_timing(self.h, 1 if on else 0), "erp_tracker_set_stage_timing")

    def stage_ms(self):
        v = [C.c_double() for _ in range(5)]
        self.ctx.check(lib().erp_tracker_stage_ms(self.h, *[C.byref(x) for x in v]), "erp_tracker_stage_ms")
        return dict(zip(["pyramids", "lk", "ransac", "gftt", "total"], [x.value for x in v]))

    def gftt_fallbacks(self):
        """(exact_tail, full_sort): downloads whose GFTT needed the masked-maximum tail / the full candidate sort"""
        a, b = C.c_int(), C.c_int()
        self.ctx.check(lib().erp_tracker_gftt_fallbacks(self.h, C.byref(a), C.byref(b)), "erp_tracker_gftt_fallbacks")
        return a.value, b.value

    def close(self):
        if self.h:
            lib().erp_tracker_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Frontend:
    """erp_frontend_*: FeatureTracker::TrackFeatures (device numerics + the reference's bookkeeping)."""

    def __init__(self, ctx, W, H, params=None):
        self.ctx = ctx
        h = C.c_void_p()
        self.params = params or default_frontend_params()
        ctx.check(lib().erp_frontend_create(ctx.h, W, H, C.byref(self.params), C.byref(h)), "erp_frontend_create")
        self.h = h
        ctx._children.add(self)

    def track(self, img):
        img = _u8img(img)
        n = C.c_int()
        self.ctx.check(lib().erp_frontend_track(self.h, _p(img), img.shape[1], C.byref(n)), "erp_frontend_track")
        ids = np.zeros(n.value, np.int32)
        xy = np.zeros((n.value, 2), np.float32)
        tc = np.zeros(n.value, np.int32)
        age = np.zeros(n.value, np.int32)
        self.ctx.check(lib().erp_frontend_features(self.h, _p(ids), _p(xy), _p(tc), _p(age), n.value),
                       "erp_frontend_features")
        nt, nd = C.c_int(), C.c_int()
        lib().erp_frontend_stats(self.h, C.byref(nt), C.byref(nd))
        return {"ids": ids, "xy": xy, "track_count": tc, "age": age, "num_tracked": nt.value, "num_detected": nd.value}

    def close(self):
        if self.h:
            lib().erp_frontend_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BaSolveCall:
    """One vio_ba_solve_batched call over fixed problems, its ctypes structs built once (Context.ba_solve_call)."""

    def __init__(self, ctx, problems, trace_cap=256):
        self.ctx = ctx
        self.problems = problems
        n = len(problems)
        self._P = (abi.VioBaProblem * n)(*[p.c for p in problems])
        self._outs = [BaOutput(p.K, p.L, p.N, trace_cap) for p in problems]
        self._O = (abi.VioBaOutput * n)(*[o.c for o in self._outs])
        self._n = n
        self._fn = lib().vio_ba_solve_batched

    def __call__(self):
        rc = self._fn(self.ctx.h, self._P, self._O, self._n)
        if rc != 0:
            self.ctx.check(rc, "vio_ba_solve_batched")

    def results(self):
        return [o.result() for o in self._outs]


class BaBatch:
    """Device-resident batch of windows (vio_ba_batch_*), for timing without host transfers."""

    def __init__(self, ctx, problems):
        self.ctx = ctx
        self.problems = problems
        n = len(problems)
        self._P = (abi.VioBaProblem * n)(*[p.c for p in problems])
        h = C.c_void_p()
        ctx.check(lib().vio_ba_batch_create(ctx.h, self._P, n, C.byref(h)), "vio_ba_batch_create")
        self.h = h
        ctx._children.add(self)

    def run(self):
        self.ctx.check(lib().vio_ba_batch_run(self.h), "vio_ba_batch_run")

    def sync(self):
        self.ctx.check(lib().vio_ba_batch_sync(self.h), "vio_ba_batch_sync")

    def set_preint(self, src, count, on_device=False):
        """vio_ba_batch_set_preint: src = (VioPreint * count) host array or a device pointer (int)."""
        ptr = src if on_device else C.cast(src, C.c_void_p)
        self.ctx.check(lib().vio_ba_batch_set_preint(self.h, ptr, int(count), 1 if on_device else 0),
                       "vio_ba_batch_set_preint")

    def kernel_ms(self):
        ms, cnt = C.c_double(), C.c_int()
        self.ctx.check(lib().vio_ba_batch_kernel_ms(self.h, C.byref(ms), C.byref(cnt)), "vio_ba_batch_kernel_ms")
        return ms.value, cnt.value

    ROUTES = {1: "phases", 2: "single-kernel", 3: "cluster"}

    def route(self):
        """vio_ba_batch_route: (route name, workgroups per window of the cluster route or 0)"""
        r, c = C.c_int(), C.c_int()
        self.ctx.check(lib().vio_ba_batch_route(self.h, C.byref(r), C.byref(c)), "vio_ba_batch_route")
        return self.ROUTES.get(r.value, str(r.value)), c.value

    PHASES = ["setup", "eval+J", "linearise", "step-prep", "schur-gemm", "cholesky", "backsub",
              "candidate", "eval-cost", "control", "post", "schur-fill", "schur-prefetch", "schur-assemble", "imu-eval", "imu-normal-eq",
              "eval-factors", "eval-landmarks", "backsub-jac", "backsub-landmarks", "backsub-candidate-cost"]

    def profile(self, enable=True):
        self.ctx.check(lib().vio_ba_batch_profile(self.h, int(enable)), "vio_ba_batch_profile")

    def phase_cycles(self):
        out = (C.c_ulonglong * 32)()
        self.ctx.check(lib().vio_ba_batch_phase_cycles(self.h, out), "vio_ba_batch_phase_cycles")
        return {n: int(out[i]) for i, n in enumerate(self.PHASES)}

    def record_bytes(self):
        """vio_ba_batch_record_bytes: the size of one packed per-window result record."""
        n = C.c_size_t()
        self.ctx.check(lib().vio_ba_batch_record_bytes(self.h, C.byref(n)), "vio_ba_batch_record_bytes")
        return n.value

    def pack(self, dst_ptr=None):
        """vio_ba_batch_pack: every window's result record; into a device buffer (int pointer, async on
        the context stream) or, with dst_ptr None, into a returned host (n, record_bytes) uint8 array."""
        if dst_ptr is not None:
            self.ctx.check(lib().vio_ba_batch_pack(self.h, dst_ptr, 1), "vio_ba_batch_pack")
            return None
        out = np.zeros((len(self.problems), self.record_bytes()), np.uint8)
        self.ctx.check(lib().vio_ba_batch_pack(self.h, _p(out), 0), "vio_ba_batch_pack")
        return out

    def download(self):
        outs = [BaOutput(p.K, p.L, p.N) for p in self.problems]
        O = (abi.VioBaOutput * len(outs))(*[o.c for o in outs])
        self.ctx.check(lib().vio_ba_batch_download(self.h, O), "vio_ba_batch_download")
        return [o.result() for o in outs]

    def close(self):
        if self.h:
            lib().vio_ba_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def ba_gather(view, variant, fix_first=True, fix_last=False):
    """vio_ba_gather (host): the Optimizer entry point's problem assembly on an abi.MapView.
    Returns the abi.GatherOut (its .result() dict, its .window(view) BaProblem window)."""
    g = abi.GatherOut(view, variant)
    rc = lib().vio_ba_gather(C.byref(view.c), int(variant), int(bool(fix_first)), int(bool(fix_last)), C.byref(g.c))
    if rc != 0:
        raise VioError(f"vio_ba_gather failed ({rc})")
    return g


def ba_write_back(view, variant, gather, out):
    """vio_ba_write_back (host): what the entry point writes into the graph, from the gather and the
    solver's BaOutput (None for a gather with status > 0).  Returns the abi.MapUpdate result dict."""
    u = abi.MapUpdate(view)
    rc = lib().vio_ba_write_back(C.byref(view.c), int(variant), C.byref(gather.c),
                                 C.byref(out.c) if out is not None else None, C.byref(u.c))
    if rc != 0:
        raise VioError(f"vio_ba_write_back failed ({rc})")
    return u.result()


class Window:
    """vio_window: the Estimator's keyframe window and MapPoint graph (CreateKeyframe slide,
    LinkMapPointsFromPreviousFrame, TriangulateNewMapPoints) on the host."""

    def __init__(self, max_keyframes=10):
        h = C.c_void_p()
        if lib().vio_window_create(int(max_keyframes), C.byref(h)):
            raise VioError("vio_window_create failed")
        self.h = h

    def close(self):
        if self.h:
            lib().vio_window_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _rc(rc, what):
        if rc:
            raise VioError(f"{what} failed ({rc})")

    def add_mappoint(self, pos, reference_frame=-1):
        p = np.ascontiguousarray(pos, np.float32).reshape(3)
        h = C.c_int32()
        self._rc(lib().vio_window_add_mappoint(self.h, _p(p), int(reference_frame), C.byref(h)), "add_mappoint")
        return h.value

    def add_observation(self, mp, frame_id, feat):
        self._rc(lib().vio_window_add_observation(self.h, int(mp), int(frame_id), int(feat)), "add_observation")

    def link_mappoints(self, prev_id, prev_valid, prev_mp, curr_id):
        pi = np.ascontiguousarray(prev_id, np.int32)
        pv = np.ascontiguousarray(prev_valid, np.uint8)
        pm = np.ascontiguousarray(prev_mp, np.int32)
        ci = np.ascontiguousarray(curr_id, np.int32)
        out = np.full(max(len(ci), 1), -1, np.int32)
        self._rc(lib().vio_window_link_mappoints(self.h, _p(pi), _p(pv), _p(pm), len(pi), _p(ci), len(ci), _p(out)),
                 "link_mappoints")
        return out[:len(ci)]

    def add_keyframe(self, frame_id, T_wb, T_bc, feature_id, bearing, valid, mappoint, uv=None, tracks=None,
                     width=960):
        """tracks: list (per feature) of [(frame_id, feature_index), ...] (Feature::GetObservations)."""
        n = len(feature_id)
        keep = [np.ascontiguousarray(T_wb, np.float32).reshape(16), np.ascontiguousarray(T_bc, np.float32).reshape(16),
                np.ascontiguousarray(feature_id, np.int32), np.ascontiguousarray(bearing, np.float32).reshape(-1),
                np.ascontiguousarray(valid, np.uint8), np.ascontiguousarray(mappoint, np.int32),
                np.ascontiguousarray(uv if uv is not None else np.zeros((n, 2)), np.float32).reshape(-1)]
        f = abi.VioWindowFrame()
        f.frame_id, f.num_features, f.width = int(frame_id), n, int(width)
        f.T_wb, f.T_bc = abi._ptr(keep[0], C.c_float), abi._ptr(keep[1], C.c_float)
        f.feature_id, f.bearing = abi._ptr(keep[2], C.c_int32), abi._ptr(keep[3], C.c_float)
        f.valid, f.mappoint, f.uv = abi._ptr(keep[4], C.c_uint8), abi._ptr(keep[5], C.c_int32), abi._ptr(keep[6], C.c_float)
        if tracks is not None:
            beg = np.zeros(n + 1, np.int32)
            fr, ft = [], []
            for i, t in enumerate(tracks):
                for (a, b) in t:
                    fr.append(a)
                    ft.append(b)
                beg[i + 1] = len(fr)
            keep += [beg, np.array(fr + [0], np.int32), np.array(ft + [0], np.int32)]
            f.track_begin, f.track_frame, f.track_feat = (abi._ptr(keep[-3], C.c_int32), abi._ptr(keep[-2], C.c_int32),
                                                          abi._ptr(keep[-1], C.c_int32))
        st = abi.VioWindowKfStats()
        self._rc(lib().vio_window_add_keyframe(self.h, C.byref(f), C.byref(st)), "add_keyframe")
        return {k: getattr(st, k) for k in ("obs_added", "transferred", "deleted", "removed_frame", "num_keyframes")}

    def triangulation_candidates(self, kf1, kf2):
        n = C.c_int()
        self._rc(lib().vio_window_triangulation_candidates(self.h, kf1, kf2, None, None, None, 0, C.byref(n)), "cand")
        m = n.value
        pairs = np.zeros((max(m, 1), 2), np.int32)
        bear = np.zeros((max(m, 1), 6), np.float32)
        T = np.zeros((2, 4, 4), np.float32)
        self._rc(lib().vio_window_triangulation_candidates(self.h, kf1, kf2, _p(pairs), _p(bear), _p(T), m, C.byref(n)),
                 "cand")
        return pairs[:m], bear[:m], T

    def commit_triangulation(self, kf1, kf2, pairs, points, valid):
        pr = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
        X = np.ascontiguousarray(points, np.float32).reshape(-1, 3)
        V = np.ascontiguousarray(valid, np.uint8)
        out = np.full(max(len(pr), 1), -1, np.int32)
        n = C.c_int()
        self._rc(lib().vio_window_commit_triangulation(self.h, kf1, kf2, _p(pr), _p(X), _p(V), len(pr), _p(out),
                                                       C.byref(n)), "commit")
        return out[:len(pr)]

    def triangulate(self, ctx, kf1, kf2):
        n = C.c_int()
        ctx.check(lib().vio_window_triangulate(self.h, ctx.h, kf1, kf2, C.byref(n)), "vio_window_triangulate")
        return n.value

    def keyframes(self):
        n = C.c_int()
        self._rc(lib().vio_window_keyframes(self.h, None, 0, C.byref(n)), "keyframes")
        out = np.zeros(max(n.value, 1), np.int32)
        self._rc(lib().vio_window_keyframes(self.h, _p(out), n.value, C.byref(n)), "keyframes")
        return out[:n.value].tolist()

    def num_mappoints(self):
        return lib().vio_window_num_mappoints(self.h)

    def mappoint(self, h):
        info = abi.VioWindowMappointInfo()
        self._rc(lib().vio_window_mappoint(self.h, int(h), C.byref(info)), "mappoint")
        n = C.c_int()
        fr = np.zeros(max(info.num_observations, 1), np.int32)
        ft = np.zeros(max(info.num_observations, 1), np.int32)
        self._rc(lib().vio_window_mappoint_observations(self.h, int(h), _p(fr), _p(ft), len(fr), C.byref(n)), "obs")
        return {"pos": np.array(info.pos, np.float32), "bad": bool(info.bad), "marg": bool(info.marginalized),
                "tri": bool(info.triangulated), "ref": info.reference_frame,
                "obs": list(zip(fr[:n.value].tolist(), ft[:n.value].tolist()))}

    def frame_mappoints(self, frame_id):
        n = C.c_int()
        self._rc(lib().vio_window_frame_mappoints(self.h, int(frame_id), None, 0, C.byref(n)), "frame_mappoints")
        out = np.zeros(max(n.value, 1), np.int32)
        self._rc(lib().vio_window_frame_mappoints(self.h, int(frame_id), _p(out), n.value, C.byref(n)), "frame_mps")
        return out[:n.value].tolist()

    def map_view(self, height=480, boundary_margin=20):
        """vio_window_map_view, copied into an abi.MapView (for ba_gather / ba_write_back)."""
        v = abi.VioMapView()
        self._rc(lib().vio_window_map_view(self.h, int(height), int(boundary_margin), C.byref(v)), "map_view")
        F, M = v.num_frames, v.num_mappoints
        a = np.ctypeslib.as_array
        G = int(a(v.feat_begin, shape=(F + 1,))[-1]) if F else 0
        nob = int(a(v.mp_obs_begin, shape=(M + 1,))[-1]) if M else 0

        def arr(ptr, n, dt):
            return a(ptr, shape=(n,)).astype(dt).copy() if n else np.zeros(0, dt)
        return abi.MapView({
            "frame_Twb": arr(v.frame_Twb, 16 * F, np.float32).reshape(-1, 4, 4),
            "frame_Tcb": arr(v.frame_Tcb, 16 * F, np.float32).reshape(-1, 4, 4),
            "feat_begin": a(v.feat_begin, shape=(F + 1,)).copy(), "feat_uv": arr(v.feat_uv, 2 * G, np.float32),
            "feat_valid": arr(v.feat_valid, G, np.uint8), "feat_mp": arr(v.feat_mp, G, np.int32),
            "mp_key": arr(v.mp_key, M, np.int64), "mp_bad": arr(v.mp_bad, M, np.uint8),
            "mp_marg": arr(v.mp_marg, M, np.uint8), "mp_pos": arr(v.mp_pos, 3 * M, np.float32),
            "mp_obs_begin": a(v.mp_obs_begin, shape=(M + 1,)).copy(), "mp_obs_frame": arr(v.mp_obs_frame, nob, np.int32),
            "mp_obs_feat": arr(v.mp_obs_feat, nob, np.int32),
            "width": v.width, "height": v.height, "boundary_margin": v.boundary_margin})

    def apply_update(self, upd):
        """vio_window_apply_update with an abi.MapUpdate (or a raw VioBaMapUpdate) of the last map view."""
        c = upd.c if hasattr(upd, "c") else upd
        self._rc(lib().vio_window_apply_update(self.h, C.byref(c)), "apply_update")
