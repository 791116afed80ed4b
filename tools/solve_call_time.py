"""Diagnostic: one config-3 (or BA_CFG=2: config-2) window, 10 fixed LM iterations -- resident batch re-run
against one vio_ba_solve_batched C-ABI call per solve (pack + one pinned upload + solve + one pinned download +
scatter) and the Python-level Context.ba_solve.  Prints ms per solve of each."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
vio = importlib.import_module("360_visual_inertial_odometry_amd")
synth = importlib.import_module("360_visual_inertial_odometry_amd.synth")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
ctx = vio.Context(0)
if os.environ.get("BA_CFG") == "2":
    p = vio.BaProblem(synth.config2(synth.SEED), variant=vio.VIO_BA_LOCAL, max_iterations=10, fixed_iterations=1)
else:
    p = vio.BaProblem(synth.config3(synth.SEED), variant=vio.VIO_BA_VI, max_iterations=10, fixed_iterations=1)
b = vio.BaBatch(ctx, [p])
for _ in range(3):
    b.run()
b.sync()
b.kernel_ms()
t0 = time.perf_counter()
for _ in range(reps):
    b.run()
b.sync()
res_ms = (time.perf_counter() - t0) / reps * 1e3
k_ms, _ = b.kernel_ms()
b.close()
call = ctx.ba_solve_call([p])
for _ in range(3):
    call()
t0 = time.perf_counter()
for _ in range(reps):
    call()
call_ms = (time.perf_counter() - t0) / reps * 1e3
t0 = time.perf_counter()
for _ in range(reps // 4):
    ctx.ba_solve([p])
py_ms = (time.perf_counter() - t0) / (reps // 4) * 1e3
print(f"cfg={os.environ.get('BA_CFG', '3')} resident_ms={res_ms:.4f} kernel_ms={k_ms:.4f} call_ms={call_ms:.4f} "
      f"python_call_ms={py_ms:.4f} call/resident={res_ms / call_ms:.3f} it/s resident={10 / res_ms * 1e3:.0f} "
      f"call={10 / call_ms * 1e3:.0f}", flush=True)
ctx.close()
