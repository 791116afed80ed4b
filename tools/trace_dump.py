"""Diagnostic: Summary::iterations traces of the HIP solver (both execution routes) and of the CPU
oracle plus a cloud of input-perturbed oracle runs, for the config-3 VI window at the reference
options and at fixed iterations.  Writes gpurun_out/trace_<route>.npz (analysed on the CPU)."""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401  (shared HIP runtime, loaded first)

vio = importlib.import_module("360_visual_inertial_odometry_amd")
synth = importlib.import_module("360_visual_inertial_odometry_amd.synth")
import oracle_lib  # noqa: E402

route = sys.argv[1] if len(sys.argv) > 1 else "phases"
ctx = vio.Context(0)
out = {}
cases = {"cfg3_ref": (synth.config3(), {}), "cfg3_fix30": (synth.config3(), dict(max_iterations=30, fixed_iterations=1)),
         "vik6_fix40": (synth.make_window(K=6, L=80, seed=5, imu=True), dict(max_iterations=40, fixed_iterations=1))}
for name, (w, kw) in cases.items():
    p = vio.BaProblem(w, variant=vio.VIO_BA_VI, **kw)
    if route == "mono":  # 33 copies: above the phase-route batch size, solved by ba_window_kernel
        g = ctx.ba_solve([p] * 33)[0]
    else:
        g = ctx.ba_solve([p])[0]
    for k, v in g["trace"].items():
        out[f"{name}/gpu/{k}"] = v
    for k in ("T_wb", "lm_xyz", "vel", "bg", "ba"):
        out[f"{name}/gpu/x_{k}"] = g[k]
    out[f"{name}/gpu/iterations"] = g["iterations"]
    print(name, route, "gpu iterations", g["iterations"], "final", g["final_cost"], flush=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"trace_{route}.npz"), **out)
ctx.close()
