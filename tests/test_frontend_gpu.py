"""GPU parity of erp_frontend (FeatureTracker::TrackFeatures: device LK / RANSAC / GFTT + host
bookkeeping) against tests/frontend_oracle.py over a rotating-camera ERP sequence: tracked-feature
id lists, positions, track counts, ages and GetTrackingStats must be identical (bitwise)."""
import numpy as np
import pytest

from frontend_oracle import FrontendOracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("clustered", [1, 0])
def test_frontend_sequence(vio, synth, gpu_ctx, clustered):
    W, H = 960, 480
    prm = vio.default_frontend_params(seed=11)
    prm.remove_clustered = clustered
    fe = vio.Frontend(gpu_ctx, W, H, prm)
    orc = FrontendOracle(vio, W, H, prm)
    carried = 0
    for f in range(6):
        img = synth.render_erp(W, H, synth.rot_yaw_pitch(1.2 * f, 0.3 * f))
        g = fe.track(img)
        o = orc.track(img)
        assert np.array_equal(g["ids"], o["ids"]), f
        assert np.array_equal(g["xy"], o["xy"]), f
        assert np.array_equal(g["track_count"], o["track_count"]) and np.array_equal(g["age"], o["age"]), f
        assert (g["num_tracked"], g["num_detected"]) == (o["num_tracked"], o["num_detected"]), f
        if f:
            carried += int((g["track_count"] > 0).sum())
    fe.close()
    assert carried > 500  # features really are carried across frames
