"""CPU checks of the dataset formats through the C-ABI — LoadCameraTimestamps /
LoadIMUData (app/main.cpp:30-90) — and of the INTER_AREA oracle (oracle/resize_oracle.py)."""
import importlib.util
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_resize_oracle():
    spec = importlib.util.spec_from_file_location("resize_oracle", os.path.join(ROOT, "oracle", "resize_oracle.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_camera_timestamps_rules(vio, tmp_path):
    p = tmp_path / "cam_timestamps.txt"
    p.write_text("0.1\n\n  0.2\nabc\n0.3xyz\n1e3\n\r\n12345.678901234\n")
    t = vio.load_camera_timestamps(str(p))
    np.testing.assert_array_equal(t, [0.1, 0.2, 0.3, 1000.0, 12345.678901234])


def test_imu_csv_rules(vio, tmp_path):
    p = tmp_path / "imu_data.csv"
    p.write_text("\n".join([
        "0.0,1,2,3,4,5,6",                 # first line: always the header, skipped
        "0.005,0.1,0.2,9.81,0.01,0.02,0.03",
        "",
        "0.010,0.1,0.2,9.81,0.01,0.02",    # 6 fields
        "0.015,0.1,x,9.81,0.01,0.02,0.03",  # bad field
        "0.020,0.1,0.2,9.81,0.01,0.02,0.03,",  # trailing comma: still 7 fields
        "0.025,0.1,0.2,1e40,0.01,0.02,0.03",   # f32 overflow (std::stof throws)
        "0.030, 0.5 ,0.2,9.81,0.01,0.02,0.03\r",  # spaces / CR
    ]) + "\n")
    d = vio.load_imu_csv(str(p))
    np.testing.assert_array_equal(d["timestamp"], [0.005, 0.020, 0.030])
    np.testing.assert_array_equal(d["ax"], np.float32([0.1, 0.1, 0.5]))
    np.testing.assert_array_equal(d["gz"], np.float32([0.03] * 3))


def test_imu_csv_round_trip(vio, synth, tmp_path):
    s = synth.imu_samples(0.0, 1.0, 200.0, np.random.default_rng(0), 1e-3, 1e-2, np.array([0, 0, -9.81]))
    f32 = s[:, 1:].astype(np.float32)
    p = tmp_path / "imu.csv"
    with open(p, "w") as f:
        f.write("timestamp,ax,ay,az,gx,gy,gz\n")
        for i in range(len(s)):
            f.write(repr(float(s[i, 0])) + "," + ",".join(repr(float(v)) for v in f32[i]) + "\n")
    d = vio.load_imu_csv(str(p))
    assert len(d) == len(s)
    np.testing.assert_array_equal(d["timestamp"], s[:, 0])
    for k, name in enumerate(("ax", "ay", "az", "gx", "gy", "gz")):
        np.testing.assert_array_equal(d[name], f32[:, k])


def test_missing_file(vio, tmp_path):
    with pytest.raises(vio.VioError):
        vio.load_imu_csv(str(tmp_path / "nope.csv"))


def test_resize_oracle_closed_forms():
    ro = load_resize_oracle()
    img = np.repeat(np.repeat(np.arange(12, dtype=np.uint8).reshape(3, 4) * 20, 4, 0), 4, 1)
    np.testing.assert_array_equal(ro.resize_area(img, 4, 3), np.arange(12, dtype=np.uint8).reshape(3, 4) * 20)
    # a 4x4 block with k ones: round-half-even(k / 16) — 8 -> 0 (0.5 to even), 24/16=1.5 -> 2
    for k, want in [(7, 0), (8, 0), (9, 1), (24, 2)]:
        b = np.zeros(16, np.uint8)
        b[:min(k, 16)] = 1 if k <= 16 else 0
        if k > 16:
            b[:] = 1
            b[:k - 16] = 2
        assert ro.resize_area(b.reshape(4, 4), 1, 1)[0, 0] == want, k
    # factor 2x2 takes OpenCV's ResizeAreaFastVec: (a + b + c + d + 2) >> 2 = round half UP
    for blk, want in [((1, 1, 0, 0), 1), ((1, 0, 0, 0), 0), ((1, 1, 1, 0), 1), ((3, 3, 0, 0), 2), ((255,) * 4, 255)]:
        assert ro.resize_area(np.array(blk, np.uint8).reshape(2, 2), 1, 1)[0, 0] == want, blk
