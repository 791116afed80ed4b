"""GPU parity of vio_imu_preintegrate (csrc/imu_preint.hip) against oracle/imu_oracle.c — bitwise.

Both evaluate IMUPreintegrator::Preintegrate (src/processing/IMUPreintegrator.cpp:143-274) in f32
with the same expression order, no FMA contraction and correctly rounded sin / cos, so every f32
field and dt_total must be identical (compared with ==, so ±0 agree).
"""
import numpy as np
import pytest

import oracle_lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(vio):
    c = vio.Context(0)
    yield c
    c.close()


def _assert_same(g, o):
    (gr, gv, gc), (orc, ov, oc) = g, o
    np.testing.assert_array_equal(gv, ov)
    for k in orc:
        assert np.array_equal(gr[k], orc[k]), (k, np.argwhere(gr[k] != orc[k])[:5])
    assert np.array_equal(gc, oc)


def _stream(synth, seed, K=10):
    w = synth.make_window(K=K, L=20, seed=seed, imu=True)
    t0 = synth.KF_DT * np.arange(K - 1)
    return w["imu_samples"], t0, t0 + synth.KF_DT


def test_config3_intervals_bitwise(vio, synth, ctx):
    s, t0, t1 = _stream(synth, 20251205)
    g = ctx.imu_preintegrate(s, t0, t1)
    o = oracle_lib.imu_preintegrate(vio, s, t0, t1)
    assert g[1].all()
    _assert_same(g, o)
    assert ctx.imu_kernel_ms() > 0


def test_biases_noise_and_batch_bitwise(vio, synth, ctx):
    # one long stream, 256 windows' worth of keyframe intervals with per-interval biases
    rng = np.random.default_rng(3)
    s, _, _ = _stream(synth, 20251207, K=40)
    n = 256 * 9
    t0 = rng.uniform(0.0, 9.5, n)
    t1 = t0 + rng.choice([0.25, 0.5, 0.005, 0.0], n)
    bg = rng.normal(0, 1e-3, (n, 3)).astype(np.float32)
    ba = rng.normal(0, 1e-2, (n, 3)).astype(np.float32)
    noise = (2e-4, 3e-3, 5e-6, 2e-5)
    g = ctx.imu_preintegrate(s, t0, t1, bg, ba, noise)
    o = oracle_lib.imu_preintegrate(vio, s, t0, t1, bg, ba, noise)
    assert 0 < g[1].sum() < n  # zero-length intervals are invalid
    _assert_same(g, o)


def test_edge_cases_bitwise(vio, ctx):
    s = np.zeros((6, 7))
    s[:, 0] = [0.0, 0.0001, 0.1, 0.105, 0.105, 0.2]
    s[:, 1:4] = [0.1, -0.2, 9.81]
    s[:, 4:7] = [[0, 0, 0], [1e-9, 0, 0], [0.5, 0.1, -0.2], [0.5, 0.1, -0.2], [3.0, 0.0, 0.0], [0, 0, 0]]
    t0 = [0.0, 0.0, 0.1, 0.3, 0.105, 0.0, -1.0]
    t1 = [0.3, 0.1, 0.101, 0.4, 0.105, 0.0, 0.0]
    g = ctx.imu_preintegrate(s, t0, t1)
    o = oracle_lib.imu_preintegrate(vio, s, t0, t1)
    np.testing.assert_array_equal(g[1], [1, 1, 1, 0, 0, 0, 0])
    _assert_same(g, o)


def test_empty_inputs_and_errors(vio, ctx):
    g = ctx.imu_preintegrate(np.zeros((0, 7)), [0.0], [1.0])
    assert g[1].tolist() == [0]
    g = ctx.imu_preintegrate(np.zeros((3, 7)), [], [])
    assert len(g[1]) == 0
    s = np.zeros((3, 7))
    s[:, 0] = [0.0, 0.2, 0.1]
    with pytest.raises(vio.VioError):
        ctx.imu_preintegrate(s, [0.0], [1.0])


def test_device_preintegration_feeds_viba(vio, synth, ctx):
    """Device ΔR/ΔV/ΔP/cov replace the host producer in a config-3 VIBA window: the solve matches
    the oracle solve on the same (device-produced) factors."""
    w = synth.make_window(K=10, L=100, seed=20251205, imu=True)
    t0 = synth.KF_DT * np.arange(9)
    rec, valid, _ = ctx.imu_preintegrate(w["imu_samples"], t0, t0 + synth.KF_DT)
    assert valid.all()
    w["preint"] = [None] + [{"delta_R": rec["delta_R"][i], "delta_V": rec["delta_V"][i], "delta_P": rec["delta_P"][i],
                             "J_Rg": rec["J_Rg"][i], "J_Vg": rec["J_Vg"][i], "J_Va": rec["J_Va"][i],
                             "J_Pg": rec["J_Pg"][i], "J_Pa": rec["J_Pa"][i],
                             "cov": np.pad(rec["cov9"][i], ((0, 6), (0, 6))),
                             "gyro_bias": rec["gyro_bias"][i], "accel_bias": rec["accel_bias"][i],
                             "dt_total": float(rec["dt_total"][i])} for i in range(9)]
    p = vio.BaProblem(w, variant=vio.VIO_BA_VI)
    g = ctx.ba_solve([p])[0]
    o = oracle_lib.ba_solve(vio, p)
    assert g["success"] == o["success"] == 1
    assert np.abs(g["T_wb"][:, :3, 3] - o["T_wb"][:, :3, 3]).max() <= 1e-4
    assert np.abs(g["lm_xyz"] - o["lm_xyz"]).max() <= 1e-3
