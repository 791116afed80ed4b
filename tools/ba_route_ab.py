"""Diagnostic: window-BA routes side by side on one box -- per batch size W (config-3 VIO windows,
10 fixed LM iterations, resident batch), the HIP-event time per launch of each route and the largest
difference of its results from the phase route's (the routes sum in different fixed orders: roundoff).

    python tools/ba_route_ab.py [W ...]      (default 1 32 256)
"""
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

vio = importlib.import_module("360_visual_inertial_odometry_amd")
synth = importlib.import_module("360_visual_inertial_odometry_amd.synth")
ctx = vio.Context(0)
ROUTES = {"phases": ctx.ROUTE_PHASES, "cluster": ctx.ROUTE_CLUSTER}
reps = int(os.environ.get("AB_REPS", "30"))
for W in [int(a) for a in sys.argv[1:]] or [1, 32, 256]:
    probs = [vio.BaProblem(synth.config3(synth.SEED + i), variant=vio.VIO_BA_VI, max_iterations=10, fixed_iterations=1)
             for i in range(W)]
    res = {}
    for name, route in ROUTES.items():
        ctx.set_ba_route(route)
        b = vio.BaBatch(ctx, probs)
        for _ in range(3):
            b.run()
        b.sync()
        b.kernel_ms()
        t0 = time.perf_counter()
        for _ in range(reps):
            b.run()
        b.sync()
        wall = (time.perf_counter() - t0) / reps
        ms, _ = b.kernel_ms()
        out = b.download()
        b.close()
        res[name] = out
        d = max(np.abs(a["T_wb"] - p["T_wb"]).max() for a, p in zip(out, res["phases"]))
        dl = max(np.abs(a["lm_xyz"] - p["lm_xyz"]).max() for a, p in zip(out, res["phases"]))
        print(f"W={W:4d} {name:8s} event_ms={ms:.4f} wall_ms={wall * 1e3:.4f} "
              f"window_iters_per_s={W * 10 / (ms * 1e-3):.0f}  vs phases: dT {d:.2e} dlm {dl:.2e}", flush=True)
ctx.set_ba_route(ctx.ROUTE_AUTO)
ctx.close()
