"""MI355X-native hot path of 93won/360_visual_inertial_odometry: ERP feature tracking + sliding-window BA.

The compute path is libvio360.so (HIP kernels for gfx950 behind the C-ABI in include/vio360.h).
This module only loads it and marshals numpy buffers; there is no CPU fallback: if the library or
a GPU is missing every entry point raises.
"""
import ctypes as C
import os

import numpy as np

from . import abi
from .abi import (VIO_BA_FULL, VIO_BA_LOCAL, VIO_BA_VI, VIO_PNP, BaOutput, BaProblem,  # noqa: F401
                  default_klt_params)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VIO360_LIB") or os.path.join(_HERE, "libvio360.so")
_lib = None

EXPORTS = [
    "vio_abi_version", "vio_ctx_create", "vio_ctx_destroy", "vio_ctx_last_error",
    "vio_ba_solve", "vio_ba_solve_batched", "vio_ba_batch_create", "vio_ba_batch_run",
    "vio_ba_batch_sync", "vio_ba_batch_download", "vio_ba_batch_kernel_ms", "vio_ba_batch_destroy",
    "vio_ba_batch_profile", "vio_ba_batch_phase_cycles",
    "erp_klt_track", "erp_gftt", "erp_rot_ransac", "erp_tracker_create", "erp_tracker_upload",
    "erp_tracker_set_points", "erp_tracker_run", "erp_tracker_sync", "erp_tracker_download",
    "erp_tracker_kernel_ms", "erp_tracker_destroy",
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
    L.vio_ba_batch_destroy.argtypes = [C.c_void_p]
    L.vio_ba_batch_profile.argtypes = [C.c_void_p, C.c_int]
    L.vio_ba_batch_phase_cycles.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
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

    def check(self, rc, what):
        if rc != 0:
            raise VioError(f"{what} failed ({rc}): {lib().vio_ctx_last_error(self.h).decode()}")

    def close(self):
        if self.h:
            lib().vio_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- bundle adjustment ----
    def ba_solve(self, problems):
        """Solve a list of BaProblem windows in one launch; returns list of result dicts."""
        n = len(problems)
        P = (abi.VioBaProblem * n)(*[p.c for p in problems])
        outs = [BaOutput(p.K, p.L, p.N) for p in problems]
        O = (abi.VioBaOutput * n)(*[o.c for o in outs])
        self.check(lib().vio_ba_solve_batched(self.h, P, O, n), "vio_ba_solve_batched")
        return [o.result() for o in outs]


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

    def run(self):
        self.ctx.check(lib().vio_ba_batch_run(self.h), "vio_ba_batch_run")

    def sync(self):
        self.ctx.check(lib().vio_ba_batch_sync(self.h), "vio_ba_batch_sync")

    def kernel_ms(self):
        ms, cnt = C.c_double(), C.c_int()
        self.ctx.check(lib().vio_ba_batch_kernel_ms(self.h, C.byref(ms), C.byref(cnt)), "vio_ba_batch_kernel_ms")
        return ms.value, cnt.value

    PHASES = ["setup", "eval+J", "linearise", "step-prep", "schur-gemm", "cholesky", "backsub",
              "candidate", "eval-cost", "control", "post"]

    def profile(self, enable=True):
        self.ctx.check(lib().vio_ba_batch_profile(self.h, int(enable)), "vio_ba_batch_profile")

    def phase_cycles(self):
        out = (C.c_ulonglong * 16)()
        self.ctx.check(lib().vio_ba_batch_phase_cycles(self.h, out), "vio_ba_batch_phase_cycles")
        return {n: int(out[i]) for i, n in enumerate(self.PHASES)}

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
