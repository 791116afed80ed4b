"""Generates tests/golden/config3_cloud.json: how far the CPU oracle's converged config-3 answer moves
under roundoff-sized input changes (its "perturbation cloud").  TEST INFRASTRUCTURE: the oracle is the
checker.

Config 3 (one 10 KF x 500 LM VIO window, RunVIBA semantics, Optimizer.cpp:493-724, at the reference's
solver options: 50 iterations, Ceres function / parameter / gradient tolerances,
trust_region_minimizer.cc:740-760) is solved once as given and once per e in CLOUD with the landmark
inputs scaled by (1 + e) — 1 to 50 ulp.  The VI window is ill-conditioned near its optimum (the
preintegrated rotation covariance is never propagated, IMUPreintegrator.cpp:240-274, so the rotation
sqrt-information is 1e4): those changes move the converged poses by up to ~3e-4 m, the biases by ~6e-4
and the iteration count over 36..51.  Any valid regrouping of the floating-point sums (the GPU's
fixed-order wave reductions, a different Schur group size) moves the answer by the same kind of amount,
so tests/test_ba_gpu.py judges converged config 3 by max(SURVEY §8c bar, 2 x this cloud) per quantity.

    python tests/golden/gen_config3_cloud.py     (about 20 s)
"""
import importlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

CLOUD = tuple(s * m * x for x in (1e-15, 1e-14) for m in (1, 2, 3, 5) for s in (1, -1))


def rot_angle(Ra, Rb):
    c = (np.trace(Ra.T @ Rb) - 1.0) / 2.0
    return float(np.arccos(max(-1.0, min(1.0, c))))


def spreads(o, c):
    """per-quantity distance of a cloud member c from the unperturbed solve o"""
    K = len(o["T_wb"])
    return {
        "pos_m": float(np.abs(o["T_wb"][:, :3, 3] - c["T_wb"][:, :3, 3]).max()),
        "rot_rad": max(rot_angle(o["T_wb"][k, :3, :3], c["T_wb"][k, :3, :3]) for k in range(K)),
        "lm_m": float(np.abs(o["lm_xyz"] - c["lm_xyz"]).max()),
        "vel": float(np.abs(o["vel"] - c["vel"]).max()),
        "bg": float(np.abs(o["bg"] - c["bg"]).max()),
        "ba": float(np.abs(o["ba"] - c["ba"]).max()),
        "cost_rel": abs(o["final_cost"] - c["final_cost"]) / o["final_cost"],
        "iterations": int(c["iterations"]),
    }


def generate():
    vio = importlib.import_module("360_visual_inertial_odometry_amd")
    synth = importlib.import_module("360_visual_inertial_odometry_amd.synth")
    import oracle_lib
    w = synth.config3()
    o = oracle_lib.ba_solve(vio, vio.BaProblem(w, variant=vio.VIO_BA_VI))
    members = []
    for e in CLOUD:
        c = oracle_lib.ba_solve(vio, vio.BaProblem(dict(w, lm_xyz=w["lm_xyz"] * (1 + e)), variant=vio.VIO_BA_VI))
        members.append(dict(spreads(o, c), e=e))
    keys = ("pos_m", "rot_rad", "lm_m", "vel", "bg", "ba", "cost_rel")
    return {
        "what": "config 3 (synth.config3(), VIO_BA_VI, reference options): oracle vs oracle on landmark inputs x (1+e)",
        "oracle": {"iterations": int(o["iterations"]), "final_cost": float(o["final_cost"])},
        "members": members,
        "max": {k: max(m[k] for m in members) for k in keys},
        "iterations_range": [min([o["iterations"]] + [m["iterations"] for m in members]),
                             max([o["iterations"]] + [m["iterations"] for m in members])],
    }


if __name__ == "__main__":
    out = generate()
    with open(os.path.join(HERE, "config3_cloud.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["max"], indent=1), out["iterations_range"])
