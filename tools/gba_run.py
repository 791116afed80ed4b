"""Diagnostic: one config-5 global BA solve (1000 KF x 50k landmarks) of N fixed LM iterations; used
under rocprofv3 for per-kernel counters of the global path (chol_syrk_kernel etc.)."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

vio = importlib.import_module("360_visual_inertial_odometry_amd")
synth = importlib.import_module("360_visual_inertial_odometry_amd.synth")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 2
ctx = vio.Context(0)
p = vio.BaProblem(synth.make_global(), variant=vio.VIO_BA_FULL, max_iterations=N, fixed_iterations=1)
t0 = time.perf_counter()
r = ctx.ba_solve([p])[0]
print(f"global BA {N} iterations: {time.perf_counter() - t0:.3f} s, cost {r['initial_cost']:.4e} -> {r['final_cost']:.4e}",
      flush=True)
ctx.close()
