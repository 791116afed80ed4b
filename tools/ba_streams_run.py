"""Diagnostic: one config-4 shard (W config-3 VIO windows, 10 fixed LM iterations) split into S
sub-batches on S contexts (= S HIP streams of one device), all launched back to back; prints the
wall time per step.  Route: VIO_BA_PHASES=1 / VIO_BA_MONOLITHIC=1 in the environment."""
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
R = int(sys.argv[2]) if len(sys.argv) > 2 else 10
probs = [vio.BaProblem(synth.config3(synth.SEED + i), variant=vio.VIO_BA_VI, max_iterations=10, fixed_iterations=1)
         for i in range(W)]
for S in [int(s) for s in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 2, 4]:
    ctxs = [vio.Context(0) for _ in range(S)]
    per = W // S
    bs = [vio.BaBatch(ctxs[s], probs[s * per:(s + 1) * per]) for s in range(S)]
    for _ in range(3):
        for b in bs:
            b.run()
    for b in bs:
        b.sync()
    t0 = time.perf_counter()
    for _ in range(R):
        for b in bs:
            b.run()
    for b in bs:
        b.sync()
    wall = (time.perf_counter() - t0) / R
    route = 'phases' if os.environ.get('VIO_BA_PHASES') == '1' else 'mono' if os.environ.get('VIO_BA_MONOLITHIC') == '1' else 'auto'
    print(f"W={W} streams={S} route={route} wall_ms={wall * 1e3:.4f} window_iters_per_s={W * 10 / wall:.0f}", flush=True)
    for b in bs:
        b.close()
    for c in ctxs:
        c.close()
