"""GPU leg of the window bookkeeping: vio_window_triangulate (candidates -> device vio_triangulate ->
commit) gives the same graph as the host halves around the numpy/LAPACK oracle triangulation
(test_window.py's path): identical MapPoint handles, flags and observation lists, positions within
the triangulation bar of test_tri_gpu.py (1e-5 relative)."""
import numpy as np
import pytest

from test_tri_oracle import load_oracle
from test_window import make_sequence

pytestmark = pytest.mark.gpu


def run(vio, frames, tri_fn, max_kf=4):
    W = vio.Window(max_kf)
    prev = None
    for fr in frames:
        mp = [-1] * len(fr["fid"]) if prev is None else \
            W.link_mappoints(prev["fid"], prev["valid"], prev["mp"], fr["fid"]).tolist()
        W.add_keyframe(fr["id"], fr["T"], np.eye(4), fr["fid"], fr["bearing"], fr["valid"], mp, tracks=fr["tracks"])
        if prev is not None:
            tri_fn(W, prev["id"], fr["id"])
        prev = dict(id=fr["id"], fid=fr["fid"], valid=fr["valid"].tolist(), mp=W.frame_mappoints(fr["id"]))
    return W


def test_device_triangulation_matches_host_path(vio, gpu_ctx):
    tri = load_oracle()

    def host(W, a, b):
        pairs, bear, T = W.triangulation_candidates(a, b)
        if len(pairs):
            X, V, _ = tri.triangulate(T, np.tile([0, 1], (len(pairs), 1)), bear, 960)
            W.commit_triangulation(a, b, pairs, X.astype(np.float32), V.astype(np.uint8))

    frames = make_sequence(np.random.default_rng(3), n_frames=12, n_tracks=80, feats=60)
    Wh = run(vio, frames, host)
    Wd = run(vio, frames, lambda W, a, b: W.triangulate(gpu_ctx, a, b))
    assert Wh.keyframes() == Wd.keyframes()
    assert Wh.num_mappoints() == Wd.num_mappoints() > 0
    for h in range(Wh.num_mappoints()):
        a, b = Wh.mappoint(h), Wd.mappoint(h)
        assert (a["bad"], a["marg"], a["tri"], a["ref"], a["obs"]) == (b["bad"], b["marg"], b["tri"], b["ref"], b["obs"])
        nrm = max(float(np.linalg.norm(a["pos"])), 1e-6)
        assert np.linalg.norm(a["pos"].astype(np.float64) - b["pos"]) / nrm < 1e-5
