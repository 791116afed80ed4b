"""Diagnostic: one config-4 shard (W config-3 VIO windows, 10 fixed LM iterations) solved S times on a
resident batch; prints the average HIP-event time per launch.  Route: VIO_BA_PHASES=1 /
VIO_BA_MONOLITHIC=1 / VIO_BA_ROUTE=cluster in the environment.  Used under rocprofv3 for per-kernel statistics.
BA_CFG=2: config-2 windows (visual-only RunLocalBA, 10 KF x 200 landmarks) instead."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

vio = importlib.import_module("360_visual_inertial_odometry_amd")
synth = importlib.import_module("360_visual_inertial_odometry_amd.synth")
W = int(sys.argv[1]) if len(sys.argv) > 1 else 256
S = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ctx = vio.Context(0)
if os.environ.get("VIO_BA_ROUTE") == "cluster":  # force the cluster route (experiment)
    ctx.set_ba_route(ctx.ROUTE_CLUSTER)
if os.environ.get("BA_CFG") == "2":
    probs = [vio.BaProblem(synth.config2(synth.SEED + i), variant=vio.VIO_BA_LOCAL, max_iterations=10,
                           fixed_iterations=1) for i in range(W)]
else:
    probs = [vio.BaProblem(synth.config3(synth.SEED + i), variant=vio.VIO_BA_VI, max_iterations=10,
                           fixed_iterations=1) for i in range(W)]
b = vio.BaBatch(ctx, probs)
for _ in range(3):
    b.run()
b.sync()
b.kernel_ms()
t0 = time.perf_counter()
for _ in range(S):
    b.run()
b.sync()
wall = (time.perf_counter() - t0) / S
ms, n = b.kernel_ms()
print(f"W={W} cfg={os.environ.get('BA_CFG', '3')} route={'phases' if os.environ.get('VIO_BA_PHASES') == '1' else 'mono' if os.environ.get('VIO_BA_MONOLITHIC') == '1' else 'auto'} "
      f"event_ms={ms:.4f} wall_ms={wall * 1e3:.4f} window_iters_per_s={W * 10 / (ms * 1e-3):.0f}", flush=True)
b.close()
ctx.close()
