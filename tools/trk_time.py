"""Diagnostic: config-1 ERP tracker pipeline (3840x1920 pair, 300 corners) stage times, the same
setup as bench.py's erp_klt leg.  VIO360_LIB=tools/probe/libvio360_dbg.so prints the GFTT selection
breakdown (GFTT_DEBUG build)."""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

vio = importlib.import_module("360_visual_inertial_odometry_amd")
synth = importlib.import_module("360_visual_inertial_odometry_amd.synth")
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
W, H = 3840, 1920
ctx = vio.Context(0)
a, b, _ = synth.config1(W, H)
mask = np.zeros((H, W), np.uint8)
mask[int(np.float32(H) * np.float32(0.15)):int(np.float32(H) * np.float32(0.85)), 20:W - 20] = 255
pts = ctx.gftt(a, mask, 300, float(np.float32(0.01)), 30.0)
prm = vio.default_tracker_params(max_corners=300, seed=1)
t = vio.Tracker(ctx, W, H, max_points=512, max_corners=512)
t.upload(0, a)
t.upload(1, b)
t.set_points(pts)
for _ in range(3):
    t.run(prm)
t.sync()
stage = None
for _ in range(steps):
    t.run(prm)
    t.sync()
    s = t.stage_ms()
    stage = {k: (stage or {}).get(k, 0.0) + v / steps for k, v in s.items()}
t.set_stage_timing(False)
tot = 0.0
for _ in range(steps):
    t.run(prm)
    t.sync()
    tot += t.stage_ms()["total"] / steps
print("total_ms without stage markers", round(tot, 4), flush=True)
res = t.download()
print("stage_ms", {k: round(v, 4) for k, v in stage.items()}, flush=True)
print("kept", int(np.sum(res["status"])) if "status" in res else None, "new corners",
      len(res["corners"]) if "corners" in res else None, flush=True)
t.close()
ctx.close()
