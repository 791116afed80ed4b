"""Diagnostic: W config-3 VIO windows (10 fixed LM iterations) as P independent batches, one context (stream)
each, enqueued back to back so that their phase kernels can overlap; prints the wall time per step (all P
batches) over S steps.  Usage: python tools/ba_split_run.py W P S"""
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
P = int(sys.argv[2]) if len(sys.argv) > 2 else 2
S = int(sys.argv[3]) if len(sys.argv) > 3 else 20
probs = [vio.BaProblem(synth.config3(synth.SEED + i), variant=vio.VIO_BA_VI, max_iterations=10, fixed_iterations=1)
         for i in range(W)]
ctxs = [vio.Context(0) for _ in range(P)]
per = (W + P - 1) // P
bs = [vio.BaBatch(ctxs[p], probs[p * per:(p + 1) * per]) for p in range(P)]
for _ in range(3):
    for b in bs:
        b.run()
for b in bs:
    b.sync()
best = 1e9
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(S):
        for b in bs:
            b.run()
    for b in bs:
        b.sync()
    best = min(best, (time.perf_counter() - t0) / S)
ev = [b.kernel_ms()[0] for b in bs]
print(f"W={W} P={P} wall_ms={best * 1e3:.4f} window_iters_per_s={W * 10 / best:.0f} "
      f"per_batch_event_ms={','.join(f'{e:.3f}' for e in ev)}", flush=True)
for b in bs:
    b.close()
for c in ctxs:
    c.close()
