"""IMU initialisation: Optimizer::OptimizeIMUInit (src/optimization/Optimizer.cpp:972-1257)
over InertialGravityScaleFactor (Factors.cpp:981-1293) and BiasPriorFactor (Factors.h:366-396).

CPU: the oracle (oracle_imu_init) on a known-answer case — a stationary, tilted IMU: every factor is
exact at gravity = the body-frame gravity, zero velocities and biases (the pose blocks enter the
factor as identity, Factors.cpp:1024-1042, so the answer lives in the body frame) — and its guards.
The reference's own tests do not cover this path: parity unpinned beyond this KAT.
GPU: vio_imu_init_solve against the oracle on synthetic VIO windows and the KAT, batched."""
import numpy as np
import pytest

import oracle_lib

G = 9.81


def rot(axis, deg):
    a = np.asarray(axis, float) / np.linalg.norm(axis)
    t = np.radians(deg)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(t) * K + (1 - np.cos(t)) * K @ K


def stationary_frames(F=6, dt=0.1, tilt=(1.0, 0.5, 0.0), tilt_deg=4.0, seed=0):
    """A stationary IMU rotated by R_wb: specific force R_bw * (0, 0, +g), so the preintegrated
    dV = -g_b dt, dP = -g_b dt^2 / 2 with g_b = R_bw (0, 0, -g), dR = I."""
    rng = np.random.default_rng(seed)
    R_wb = rot(tilt, tilt_deg)
    g_b = R_wb.T @ np.array([0.0, 0.0, -G])
    T = np.tile(np.eye(4), (F, 1, 1))
    T[:, :3, :3] = R_wb
    pre = [None]
    for _ in range(1, F):
        pre.append({
            "delta_R": np.eye(3, dtype=np.float32), "delta_V": (-g_b * dt).astype(np.float32),
            "delta_P": (-0.5 * g_b * dt * dt).astype(np.float32),
            "J_Rg": (-dt * np.eye(3) + rng.normal(0, 1e-4, (3, 3))).astype(np.float32),
            "J_Vg": rng.normal(0, 1e-3, (3, 3)).astype(np.float32), "J_Va": (-dt * np.eye(3)).astype(np.float32),
            "J_Pg": rng.normal(0, 1e-4, (3, 3)).astype(np.float32),
            "J_Pa": (-0.5 * dt * dt * np.eye(3)).astype(np.float32),
            "cov": (np.eye(15) * 1e-4).astype(np.float32), "gyro_bias": np.zeros(3, np.float32),
            "accel_bias": np.zeros(3, np.float32), "dt_total": dt})
    return {"T_wb": T, "preint": pre}, g_b


def window_frames(synth, seed):
    w = synth.config3(seed)
    return {"T_wb": w["T_wb_init"], "preint": w["preint"]}


def test_oracle_stationary_kat(vio):
    fr, g_b = stationary_frames()
    r = oracle_lib.imu_init(vio, vio.abi.ImuInitProblem(fr))
    assert r["success"] == 1 and r["status"] == 0
    # gravity = R_wg (0, 0, -9.81) recovers the body-frame gravity (f32 inputs: ~1e-6)
    np.testing.assert_allclose(r["gravity"], g_b, rtol=0, atol=1e-4)
    # the quirky velocity initialisation R_wb_prev * dV = (0, 0, g dt) is matched in stage 1 by
    # scale -> 0; with scale ~ 0 the velocities are unobservable in stage 2: only s * v is pinned
    np.testing.assert_allclose(r["scale"] * r["velocities"], 0.0, atol=1e-6)
    np.testing.assert_allclose(r["gyro_bias"], 0.0, atol=1e-4)
    np.testing.assert_allclose(r["accel_bias"], 0.0, atol=1e-4)
    assert r["final_cost"] < 1e-8
    np.testing.assert_allclose(r["Rwg"] @ r["Rwg"].T, np.eye(3), atol=1e-12)


def test_oracle_guards(vio):
    fr, _ = stationary_frames(F=3)
    two = {"T_wb": fr["T_wb"][:2], "preint": fr["preint"][:2]}
    r = oracle_lib.imu_init(vio, vio.abi.ImuInitProblem(two))
    assert r["success"] == 0 and r["status"] == vio.abi.VIO_IMU_INIT_FEW_FRAMES
    assert r["scale"] == 1.0 and r["gravity"][2] == pytest.approx(-9.81, abs=1e-6)
    miss = {"T_wb": fr["T_wb"], "preint": [None, fr["preint"][1], None]}
    assert oracle_lib.imu_init(vio, vio.abi.ImuInitProblem(miss))["status"] == vio.abi.VIO_IMU_INIT_NO_PREINT
    long_dt = {"T_wb": fr["T_wb"], "preint": [None] + [dict(p, dt_total=2.5) for p in fr["preint"][1:]]}
    r = oracle_lib.imu_init(vio, vio.abi.ImuInitProblem(long_dt))
    assert r["status"] == vio.abi.VIO_IMU_INIT_NO_FACTORS and r["success"] == 0


def test_oracle_window_runs_both_stages(vio, synth):
    """A config-3 window's preintegrations: both stages run, the stage-2 cost does not exceed the
    stage-1 initial cost, the velocity initialisation R_wb_prev * delta_V feeds stage 2."""
    r = oracle_lib.imu_init(vio, vio.abi.ImuInitProblem(window_frames(synth, synth.SEED)))
    assert r["success"] == 1
    assert all(1 <= it <= 51 for it in r["iterations"])
    assert r["final_cost"] <= r["initial_cost"]
    assert abs(np.linalg.norm(r["gravity"]) - 9.81) < 1e-9


def assert_parity(g, o, tol=1e-9):
    assert g["status"] == o["status"] and g["success"] == o["success"]
    if o["status"]:
        return
    assert g["iterations"] == o["iterations"] and g["termination"] == o["termination"]
    for k in ("gravity_dir", "gyro_bias", "accel_bias", "velocities", "gravity"):
        np.testing.assert_allclose(g[k], o[k], rtol=tol, atol=tol * 10, err_msg=k)
    assert g["scale"] == pytest.approx(o["scale"], rel=tol)
    assert g["initial_cost"] == pytest.approx(o["initial_cost"], rel=tol)
    assert g["final_cost"] == pytest.approx(o["final_cost"], rel=1e-7, abs=1e-12)


@pytest.mark.gpu
def test_gpu_matches_oracle_batched(vio, synth):
    ctx = vio.Context(0)
    try:
        frames = [window_frames(synth, synth.SEED + k) for k in range(4)]
        frames += [stationary_frames(F=3 + k, seed=k)[0] for k in range(4)]
        frames.append({"T_wb": frames[0]["T_wb"][:2], "preint": frames[0]["preint"][:2]})  # guard inside a batch
        probs = [vio.abi.ImuInitProblem(f) for f in frames]
        got = ctx.imu_init(probs)
        for k, p in enumerate(probs):
            assert_parity(got[k], oracle_lib.imu_init(vio, p))
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_stationary_kat(vio):
    ctx = vio.Context(0)
    try:
        fr, g_b = stationary_frames(F=10, tilt=(0.2, -1.0, 0.3), tilt_deg=7.0)
        r = ctx.imu_init([vio.abi.ImuInitProblem(fr)])[0]
        assert r["success"] == 1
        np.testing.assert_allclose(r["gravity"], g_b, rtol=0, atol=1e-4)
    finally:
        ctx.close()
