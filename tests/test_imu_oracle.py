"""CPU checks of the IMU preintegration oracle (oracle/imu_oracle.c), SURVEY §8 f1.

Reference: IMUPreintegrator::Preintegrate / IntegrateMeasurement / UpdateCovariance
(src/processing/IMUPreintegrator.cpp:143-274).  The reference has no test for this path (Eigen is
unpinned), so the oracle is pinned by (1) the independent numpy f32 restatement in synth.py
(BLAS-ordered products: agreement to 1e-6 relative — a few f32 ulps — not bitwise), (2) closed forms, (3) the
reference's range / dt rules.
"""
import numpy as np
import pytest

import oracle_lib

F32 = np.float32


def _window_stream(synth, seed):
    w = synth.make_window(K=10, L=20, seed=seed, imu=True)
    K = 10
    t0 = np.array([synth.KF_DT * (i - 1) for i in range(1, K)])
    t1 = np.array([synth.KF_DT * i for i in range(1, K)])
    return w, t0, t1


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


@pytest.mark.parametrize("seed", [20251205, 20251206])
def test_oracle_matches_numpy_restatement(vio, synth, seed):
    w, t0, t1 = _window_stream(synth, seed)
    rec, valid, cov_bias = oracle_lib.imu_preintegrate(vio, w["imu_samples"], t0, t1)
    assert valid.all()
    for i in range(len(t0)):
        ref = w["preint"][i + 1]
        for name in ("delta_R", "delta_V", "delta_P", "J_Rg", "J_Vg", "J_Va", "J_Pg", "J_Pa"):
            assert _rel(rec[name][i], ref[name]) < 1e-6, (i, name, _rel(rec[name][i], ref[name]))
        assert _rel(rec["cov9"][i], ref["cov"][:9, :9]) < 1e-6, (i, _rel(rec["cov9"][i], ref["cov"][:9, :9]))
        assert abs(rec["dt_total"][i] - ref["dt_total"]) < 1e-9
        # the bias random walk: n steps of (σ_b²)·dt
        np.testing.assert_allclose(cov_bias[i], np.diag(ref["cov"])[9:], rtol=1e-5)


def _const_stream(T=0.25, rate=200.0, acc=(0.3, -0.2, 9.81), gyr=(0.0, 0.0, 0.0)):
    ts = np.arange(int(round(T * rate)) + 1) / rate
    s = np.zeros((len(ts), 7))
    s[:, 0] = ts
    s[:, 1:4] = acc
    s[:, 4:7] = gyr
    return s


def test_constant_acceleration_closed_form(vio):
    a = np.array([0.3, -0.2, 9.81])
    s = _const_stream(acc=a)
    rec, valid, _ = oracle_lib.imu_preintegrate(vio, s, [0.0], [0.25])
    assert valid[0] == 1
    n = 50  # samples in [0, 0.25)
    T = rec["dt_total"][0]
    assert abs(T - n * float(F32(0.005))) < 1e-12
    assert np.array_equal(rec["delta_R"][0], np.eye(3, dtype=F32))  # ω = 0: small-angle branch, exact
    np.testing.assert_allclose(rec["delta_V"][0], a * T, rtol=2e-6)
    np.testing.assert_allclose(rec["delta_P"][0], 0.5 * a * T * T, rtol=2e-5)
    np.testing.assert_allclose(rec["J_Va"][0], np.eye(3) * T, rtol=2e-6, atol=0)
    # J_Pa accumulates the *updated* J_Va (IMUPreintegrator.cpp:235): Σ_k (k·dt² + ½dt²) = ½T² + T·dt
    dt = float(F32(0.005))
    np.testing.assert_allclose(rec["J_Pa"][0], np.eye(3) * (0.5 * T * T + T * dt), rtol=2e-5, atol=0)
    np.testing.assert_allclose(rec["J_Rg"][0], -np.eye(3) * float(F32(0.005)), rtol=1e-7, atol=0)
    # cov9: rotation rows / columns stay zero (B has no gyro columns, IMUPreintegrator.cpp:259-263)
    assert not rec["cov9"][0][:3, :].any() and not rec["cov9"][0][:, :3].any()
    c = rec["cov9"][0]
    np.testing.assert_allclose(c, c.T, rtol=1e-5, atol=1e-20)
    # velocity block: Σ n · σ_a² dt² I (ΔR = I)
    np.testing.assert_allclose(np.diag(c)[3:6], n * 1e-6 * float(F32(0.005)) ** 2, rtol=1e-4)


def test_constant_rotation_closed_form(vio, synth):
    w = np.array([0.1, -0.3, 0.8])
    s = _const_stream(acc=(0.0, 0.0, 0.0), gyr=w)
    rec, _, _ = oracle_lib.imu_preintegrate(vio, s, [0.0], [0.25])
    T = rec["dt_total"][0]
    np.testing.assert_allclose(rec["delta_R"][0], synth.so3_exp(w * T), atol=2e-6)
    assert not rec["delta_V"][0].any() and not rec["delta_P"][0].any()


def test_bias_is_subtracted(vio):
    b = np.array([0.01, -0.02, 0.03], np.float32)
    s = _const_stream(acc=(1.0, 2.0, 3.0), gyr=b)
    rec, _, _ = oracle_lib.imu_preintegrate(vio, s, [0.0], [0.25], gyro_bias=b, accel_bias=[1.0, 2.0, 3.0])
    assert np.array_equal(rec["delta_R"][0], np.eye(3, dtype=F32))
    assert not rec["delta_V"][0].any()
    np.testing.assert_array_equal(rec["gyro_bias"][0], b)


def test_range_and_dt_rules(vio):
    # samples at 0, 0.001 (dup-ish: clamps to 0.5 ms), 0.1 (gap: clamps to 20 ms), 0.105, 0.105 (dup)
    s = np.zeros((5, 7))
    s[:, 0] = [0.0, 0.0001, 0.1, 0.105, 0.105]
    s[:, 3] = 9.81
    t0 = [0.0, 0.0, 0.1, 0.2, 0.105, 0.0]
    t1 = [0.2, 0.1, 0.101, 0.3, 0.105, 0.0]  # full, half-open end, single sample, empty, empty, empty
    rec, valid, _ = oracle_lib.imu_preintegrate(vio, s, t0, t1)
    np.testing.assert_array_equal(valid, [1, 1, 1, 0, 0, 0])
    c = lambda x: float(F32(x))  # noqa: E731
    # first dt = t1 - t0 of the filtered list (clamped), then successive differences (clamped)
    full = c(max(F32(0.0005), F32(0.0001))) * 2 + c(0.02) + c(0.005) + c(0.0005)
    assert abs(rec["dt_total"][0] - full) < 1e-12
    assert abs(rec["dt_total"][1] - 2 * c(0.0005)) < 1e-12   # 0.1 excluded (t < t_end)
    assert abs(rec["dt_total"][2] - c(0.002)) < 1e-12         # one sample: dt = 0.002
    assert not rec["dt_total"][3:].any() and not rec["delta_R"][3:].any()


def test_unsorted_samples_rejected(vio):
    s = _const_stream()
    s[[3, 4]] = s[[4, 3]]
    with pytest.raises(RuntimeError):
        oracle_lib.imu_preintegrate(vio, s, [0.0], [0.25])
