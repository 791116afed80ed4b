"""GPU parity of vio_imu_preintegrate (csrc/imu_preint.hip) against oracle/imu_oracle.c — bitwise.

Both evaluate IMUPreintegrator::Preintegrate (src/processing/IMUPreintegrator.cpp:143-274) in f32
with the same expression order, no FMA contraction and correctly rounded sin / cos, so every f32
field and dt_total must be identical (compared with ==, so ±0 agree).
"""
import ctypes as C

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


def _as_dicts(rec, K):
    return [None] + [{"delta_R": rec["delta_R"][k], "delta_V": rec["delta_V"][k], "delta_P": rec["delta_P"][k],
                      "J_Rg": rec["J_Rg"][k], "J_Vg": rec["J_Vg"][k], "J_Va": rec["J_Va"][k],
                      "J_Pg": rec["J_Pg"][k], "J_Pa": rec["J_Pa"][k], "cov": np.pad(rec["cov9"][k], ((0, 6), (0, 6))),
                      "gyro_bias": rec["gyro_bias"][k], "accel_bias": rec["accel_bias"][k],
                      "dt_total": float(rec["dt_total"][k])} for k in range(1, K)]


def test_device_preintegration_chain_into_batch(vio, synth, ctx):
    """vio_imu_preintegrate_device writes each window's factors straight into device memory,
    vio_ba_batch_set_preint moves them into a VIBA batch (no host round trip); the solve is bitwise
    the solve of a batch created with the same factors from the host."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    K, nw = 10, 4
    ws = [synth.make_window(K=K, L=60, seed=20251230 + w, imu=True) for w in range(nw)]
    t0 = np.r_[-1.0, synth.KF_DT * np.arange(K - 1)]  # entry 0: empty range -> invalid, unused
    t1 = np.r_[-1.0, synth.KF_DT * np.arange(1, K)]
    sz = C.sizeof(vio.abi.VioPreint)
    d_out = torch.zeros(nw * K * sz, dtype=torch.uint8, device=dev)
    d_valid = torch.zeros(nw * K, dtype=torch.uint8, device=dev)
    d_cov = torch.zeros(nw * K * 6, dtype=torch.float32, device=dev)
    d_t0 = torch.from_numpy(t0).to(dev)
    d_t1 = torch.from_numpy(t1).to(dev)
    keep = []
    host_recs = []
    for w, win in enumerate(ws):
        imu = vio.abi.imu_array(win["imu_samples"])
        d_imu = torch.from_numpy(imu.view(np.uint8).copy()).to(dev)
        keep.append(d_imu)
        torch.cuda.synchronize()
        ctx.imu_preintegrate_device(d_imu.data_ptr(), len(imu), d_t0.data_ptr(), d_t1.data_ptr(), K,
                                    d_out.data_ptr() + w * K * sz, d_valid.data_ptr() + w * K,
                                    d_cov.data_ptr() + w * K * 24)
        ctx.imu_kernel_ms()  # waits
        rec, valid, _ = ctx.imu_preintegrate(imu, t0, t1)
        assert valid.tolist() == [0] + [1] * (K - 1)
        host_recs.append(rec)
    raw = d_out.cpu().numpy()
    for w in range(nw):  # the device buffer is bitwise the host entry's output
        got = vio.abi.preint_records((vio.abi.VioPreint * K).from_buffer_copy(raw[w * K * sz:(w + 1) * K * sz].tobytes()))
        for k in got:
            assert np.array_equal(got[k], host_recs[w][k]), k
    # batch A: created from the numpy-restated factors, then overwritten on device
    pa = [vio.BaProblem(win, variant=vio.VIO_BA_VI) for win in ws]
    A = vio.BaBatch(ctx, pa)
    A.set_preint(d_out.data_ptr(), nw * K, on_device=True)
    A.run()
    A.sync()
    ra = A.download()
    # batch B: created directly from the same factors
    for w, win in enumerate(ws):
        win["preint"] = _as_dicts(host_recs[w], K)
    pb = [vio.BaProblem(win, variant=vio.VIO_BA_VI) for win in ws]
    B = vio.BaBatch(ctx, pb)
    B.run()
    B.sync()
    rb = B.download()
    for a, b in zip(ra, rb):
        assert a["success"] == b["success"] == 1
        assert np.array_equal(a["T_wb"], b["T_wb"]) and np.array_equal(a["lm_xyz"], b["lm_xyz"])
        assert a["final_cost"] == b["final_cost"]
    A.close()
    B.close()
    with pytest.raises(vio.VioError):
        vio.BaBatch(ctx, pb[:1]).set_preint(d_out.data_ptr(), 3, on_device=True)
