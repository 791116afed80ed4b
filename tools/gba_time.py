"""Diagnostic: config-5 global BA per-LM-iteration time (2L - L iteration solves, as bench.py)."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

vio = importlib.import_module("360_visual_inertial_odometry_amd")
synth = importlib.import_module("360_visual_inertial_odometry_amd.synth")
L = int(sys.argv[1]) if len(sys.argv) > 1 else 5
ctx = vio.Context(0)
w = synth.make_global()
p = vio.BaProblem(w, variant=vio.VIO_BA_FULL, max_iterations=L, fixed_iterations=1)
p2 = vio.BaProblem(w, variant=vio.VIO_BA_FULL, max_iterations=2 * L, fixed_iterations=1)
ctx.ba_solve([p])
t0 = time.perf_counter()
ctx.ba_solve([p])
a = time.perf_counter() - t0
t0 = time.perf_counter()
ctx.ba_solve([p2])
b = time.perf_counter() - t0
print(f"gba split={'off' if os.environ.get('VIO_GBA_NO_CU_SPLIT') else 'on'} ms_per_iteration={(b - a) / L * 1e3:.3f}", flush=True)
ctx.close()
