"""Diagnostic: per-phase shader-clock breakdown of the window solver for W windows (default route for the
batch size; VIO_BA_PHASES=1 forces the phase kernels).  Cluster-route slots: 8-12, 23."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

vio = importlib.import_module("360_visual_inertial_odometry_amd")
synth = importlib.import_module("360_visual_inertial_odometry_amd.synth")
W = int(sys.argv[1]) if len(sys.argv) > 1 else 1
ctx = vio.Context(0)
probs = [vio.BaProblem(synth.config3(synth.SEED + i), variant=vio.VIO_BA_VI, max_iterations=10, fixed_iterations=1)
         for i in range(W)]
b = vio.BaBatch(ctx, probs)
print("route", b.route())
b.profile(True)
b.run(); b.sync()
import ctypes as C
out = (C.c_ulonglong * 32)()
ctx.check(vio.lib().vio_ba_batch_phase_cycles(b.h, out), "phase_cycles")
names = {0: "prep U partials", 1: "prep imu", 2: "prep cost partials", 3: "prep imu normal eq", 4: "prep gradient",
         5: "prep finalize+diag", 6: "schur g0 landmark blocks", 15: "schur g0 zero panel", 7: "schur g0 fills",
         13: "schur g0 mfma phases", 14: "schur g0 combine+write", 8: "chol diag / cl leader wait A", 9: "chol panels / cl leader wait B", 10: "chol trailing / cl leader imu",
         11: "chol forward / cl member1 wait R",
         12: "chol backward / cl member1 wait F", 23: "cl member1 walk",
         16: "solve assembly+partials", 17: "solve cholesky+solves", 18: "solve small inputs+tables",
         19: "solve pose tiles+partials", 20: "solve reductions", 21: "ctrl lane", 22: "ctrl copies",
         24: "cl imu loads", 25: "cl imu model change", 26: "cl imu factors", 27: "cl imu cost", 28: "cl imu normal eq",
         29: "solve mode-1 head (loads)", 30: "solve mode-2 head (partials)", 25: "solve mode-2 fail flags",
         31: "cl member1 walk head (to back-sub)"}
tot = sum(out[i] for i in names)
for i, n in names.items():
    print(f"W={W} {n:28s} cycles/window/iter {out[i] / W / 11:10.0f}  ({100 * out[i] / max(tot, 1):.1f}%)")
b.close(); ctx.close()
