"""Diagnostic: solve W config-3 windows (10 fixed LM iterations, default route for the batch size) and print
a SHA-256 over every window's outputs -- for bitwise A/B of two builds or environment settings
(e.g. VIO_BA_IMU_BACK_MAX=0 against the default: IMU normal equations formed by ph_prep or speculatively).
usage: python tools/ba_result_hash.py W"""
import hashlib
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

vio = importlib.import_module("360_visual_inertial_odometry_amd")
synth = importlib.import_module("360_visual_inertial_odometry_amd.synth")
W = int(sys.argv[1]) if len(sys.argv) > 1 else 32
ctx = vio.Context(0)
probs = [vio.BaProblem(synth.config3(synth.SEED + i), variant=vio.VIO_BA_VI, max_iterations=10, fixed_iterations=1)
         for i in range(W)]
res = ctx.ba_solve(probs)
h = hashlib.sha256()
for r in res:
    for key in ("T_wb", "lm_xyz", "obs_chi2", "vel", "bg", "ba"):
        h.update(np.ascontiguousarray(r[key]).tobytes())
    h.update(repr((r["final_cost"], r["iterations"])).encode())
print(f"W={W} imu_back_max={os.environ.get('VIO_BA_IMU_BACK_MAX', 'default')} sha256={h.hexdigest()}")
ctx.close()
