"""CPU checks of the Estimator window bookkeeping (vio_window_*, csrc/window_host.cpp)
against a Python restatement of the reference's rules, written from src/processing/Estimator.cpp
(CreateKeyframe :671-754, LinkMapPointsFromPreviousFrame :806-843, TriangulateNewMapPoints
:1141-1318) and src/database/MapPoint.cpp (AddObservation :51-69, RemoveObservation :71-89,
IsObservedByFrame :91-104).  Random keyframe sequences with feature tracks; the triangulation between
the two bookkeeping halves is the numpy oracle (tests/tri_cases / oracle/tri_oracle.py).  The GPU leg
(vio_window_triangulate, the device kernel in between) is in test_window_gpu.py."""
import numpy as np
import pytest

from test_tri_oracle import load_oracle


class PyMap:
    def __init__(self, pos, ref=-1):
        self.pos = np.array(pos, np.float32)
        self.bad = self.marg = self.tri = False
        self.ref = ref
        self.obs = []

    def add(self, fid, feat):  # MapPoint::AddObservation
        for o in self.obs:
            if o[0] == fid:
                o[1] = feat
                return
        self.obs.append([fid, feat])

    def remove(self, fid):  # MapPoint::RemoveObservation
        self.obs = [o for o in self.obs if o[0] != fid]
        if not self.obs:
            self.bad = True

    def observed(self, fid):
        return any(o[0] == fid for o in self.obs)


class PyWindow:
    def __init__(self, max_kf):
        self.max_kf, self.frames, self.win, self.mps = max_kf, {}, [], []

    def good(self, h):
        return h >= 0 and not self.mps[h].bad

    def link(self, prev_id, prev_valid, prev_mp, curr_id):
        m = {}
        for i, (f, v) in enumerate(zip(prev_id, prev_valid)):
            if v:
                m[f] = i
        return [prev_mp[m[f]] if f in m and self.good(prev_mp[m[f]]) else -1 for f in curr_id]

    def add_keyframe(self, fr):
        fr = dict(fr, mp=list(fr["mp"]))
        self.frames[fr["id"]] = fr
        self.win.append(fr["id"])
        st = dict(obs_added=0, transferred=0, deleted=0, removed_frame=-1)
        for i, h in enumerate(fr["mp"]):
            if self.good(h) and fr["valid"][i] and not self.mps[h].observed(fr["id"]):
                self.mps[h].add(fr["id"], i)
                st["obs_added"] += 1
        while len(self.win) > self.max_kf:
            old = self.frames[self.win[0]]
            for h in old["mp"]:
                if not self.good(h) or self.mps[h].ref != old["id"]:
                    continue
                nref = next((k for k in self.win[1:] if self.mps[h].observed(k)), None)
                if nref is not None:
                    self.mps[h].ref, self.mps[h].marg = nref, True
                    st["transferred"] += 1
                else:
                    self.mps[h].bad = True
                    st["deleted"] += 1
            for h in old["mp"]:
                if self.good(h):
                    self.mps[h].remove(old["id"])
            st["removed_frame"] = old["id"]
            self.win.pop(0)
        st["num_keyframes"] = len(self.win)
        return st

    def candidates(self, k1, k2):
        a, b = self.frames[k1], self.frames[k2]
        m1 = {}
        for i, (f, v) in enumerate(zip(a["fid"], a["valid"])):
            if v:
                m1[f] = i
        out = []
        for i2, (f, v) in enumerate(zip(b["fid"], b["valid"])):
            if v and f in m1 and not self.good(b["mp"][i2]):
                out.append((m1[f], i2))
        return out

    def commit(self, k1, k2, pairs, X, valid):
        a, b = self.frames[k1], self.frames[k2]
        for (i1, i2), x, v in zip(pairs, X, valid):
            if not v:
                continue
            m = PyMap(x, k1)
            m.tri = True
            self.mps.append(m)
            h = len(self.mps) - 1
            m.add(k1, i1)
            m.add(k2, i2)
            a["mp"][i1] = h
            b["mp"][i2] = h
            for (oid, idx) in b["tracks"][i2]:
                if oid in (k1, k2) or oid not in self.frames or oid not in self.win:
                    continue
                if idx < 0 or idx >= len(self.frames[oid]["fid"]):
                    continue
                m.add(oid, idx)
                self.frames[oid]["mp"][idx] = h


def compare(vio, W, P):
    assert W.keyframes() == P.win
    assert W.num_mappoints() == len(P.mps)
    for h, m in enumerate(P.mps):
        g = W.mappoint(h)
        assert (g["bad"], g["marg"], g["tri"], g["ref"]) == (m.bad, m.marg, m.tri, m.ref), h
        assert g["obs"] == [tuple(o) for o in m.obs], h
        assert np.array_equal(g["pos"], m.pos)
    for fid in P.frames:
        assert W.frame_mappoints(fid) == P.frames[fid]["mp"], fid


def make_sequence(rng, n_frames=16, n_tracks=60, feats=40):
    """Keyframes with feature tracks: each track lives over a random span of frames."""
    life = {t: (int(rng.integers(0, n_frames)), int(rng.integers(2, 8))) for t in range(n_tracks)}
    frames, tracks_so_far = [], {}
    for f in range(n_frames):
        alive = [t for t, (s, L) in life.items() if s <= f < s + L]
        rng.shuffle(alive)
        alive = alive[:feats]
        # duplicate feature ids now and then (the reference's unordered_map keeps the last)
        if len(alive) > 3 and rng.random() < 0.3:
            alive.append(alive[0])
        n = len(alive)
        b = rng.normal(size=(n, 3))
        b /= np.linalg.norm(b, axis=1, keepdims=True)
        valid = (rng.random(n) > 0.1).astype(np.uint8)
        T = np.eye(4, dtype=np.float32)
        T[:3, 3] = [0.2 * f, 0.01 * f, 0.0]
        tracks = [list(tracks_so_far.get(t, [])) for t in alive]
        for i, t in enumerate(alive):
            tracks_so_far.setdefault(t, []).append((100 + f, i))
        frames.append(dict(id=100 + f, fid=alive, bearing=b.astype(np.float32), valid=valid, T=T, tracks=tracks))
    return frames


@pytest.mark.parametrize("seed,max_kf", [(0, 4), (1, 10), (2, 3)])
def test_window_sequence_matches_restatement(vio, seed, max_kf):
    rng = np.random.default_rng(seed)
    tri = load_oracle()
    W, P = vio.Window(max_kf), PyWindow(max_kf)
    frames = make_sequence(rng)
    T_bc = np.eye(4, dtype=np.float32)
    prev = None
    # a few initial MapPoints (Initializer::CreateMapPoints: no reference keyframe)
    for j in range(5):
        pos = rng.normal(size=3).astype(np.float32)
        assert W.add_mappoint(pos) == j
        P.mps.append(PyMap(pos))
    for fr in frames:
        n = len(fr["fid"])
        if prev is None:
            mp = [-1] * n
            if n > 5:
                mp[:5] = range(5)
        else:
            mp = P.link(prev["fid"], prev["valid"], prev["mp"], fr["fid"])
            got = W.link_mappoints(prev["fid"], prev["valid"], prev["mp"], fr["fid"])
            assert got.tolist() == mp
        st = W.add_keyframe(fr["id"], fr["T"], T_bc, fr["fid"], fr["bearing"], fr["valid"], mp, tracks=fr["tracks"])
        pst = P.add_keyframe(dict(id=fr["id"], fid=fr["fid"], valid=fr["valid"].tolist(), mp=mp, tracks=fr["tracks"]))
        assert st == pst
        compare(vio, W, P)
        if prev is not None:
            pairs, bear, T = W.triangulation_candidates(prev["id"], fr["id"])
            assert [tuple(p) for p in pairs.tolist()] == P.candidates(prev["id"], fr["id"])
            if len(pairs):
                X, V, _ = tri.triangulate(T, np.tile([0, 1], (len(pairs), 1)), bear, 960)
                V = V.astype(np.uint8)
                V[::7] = 0  # a few failed triangulations
                W.commit_triangulation(prev["id"], fr["id"], pairs, X.astype(np.float32), V)
                P.commit(prev["id"], fr["id"], [tuple(p) for p in pairs.tolist()], X.astype(np.float32), V)
            compare(vio, W, P)
        prev = dict(id=fr["id"], fid=fr["fid"], valid=fr["valid"].tolist(), mp=W.frame_mappoints(fr["id"]))
    assert any(m.marg for m in P.mps) and any(m.bad for m in P.mps)


def test_map_view_feeds_gather_and_write_back(vio):
    """The window's map view is a valid vio_map_view: RunLocalBA's gather over it sees the window's
    good MapPoints and the observations of in-window keyframes; a write-back applied to the window
    moves its poses / positions."""
    rng = np.random.default_rng(5)
    W = vio.Window(4)
    frames = make_sequence(rng, n_frames=6, n_tracks=30, feats=25)
    tri = load_oracle()
    prev = None
    for fr in frames:
        mp = [-1] * len(fr["fid"]) if prev is None else \
            W.link_mappoints(prev["fid"], prev["valid"], prev["mp"], fr["fid"]).tolist()
        uv = np.stack([rng.uniform(100, 800, len(mp)), rng.uniform(100, 380, len(mp))], 1)
        W.add_keyframe(fr["id"], fr["T"], np.eye(4), fr["fid"], fr["bearing"], fr["valid"], mp, uv=uv,
                       tracks=fr["tracks"])
        if prev is not None:
            pairs, bear, T = W.triangulation_candidates(prev["id"], fr["id"])
            if len(pairs):
                X, V, _ = tri.triangulate(T, np.tile([0, 1], (len(pairs), 1)), bear, 960)
                W.commit_triangulation(prev["id"], fr["id"], pairs, X.astype(np.float32), V.astype(np.uint8))
        prev = dict(id=fr["id"], fid=fr["fid"], valid=fr["valid"].tolist(), mp=W.frame_mappoints(fr["id"]))
    v = W.map_view()
    assert v.F == 4 and v.M == W.num_mappoints()
    g = vio.ba_gather(v, vio.VIO_BA_LOCAL).result()
    assert g["status"] == 0 and len(g["lm_mp"]) > 0
    good = [h for h in range(W.num_mappoints()) if not W.mappoint(h)["bad"]]
    assert set(g["lm_mp"].tolist()) <= set(good)
    u = vio.abi.MapUpdate(v)
    u.frame_Twb[:] = np.tile(np.eye(4, dtype=np.float32), (v.F, 1, 1)).reshape(-1)
    u.frame_Twb[3::16] = 7.0
    u.frame_set[:] = 1
    u.mp_pos[:] = 3.0
    u.mp_set[good[0]] = 1
    u.mp_set_bad[good[1]] = 1
    W.apply_update(u)
    assert np.array_equal(W.mappoint(good[0])["pos"], [3.0, 3.0, 3.0])
    assert W.mappoint(good[1])["bad"]
    assert W.map_view().frame_Twb[3] == 7.0


def test_add_keyframe_rejects_malformed_track_offsets(vio):
    """vio_window_add_keyframe checks the caller's CSR feature-track offsets (track_begin monotonic)
    before any later triangulation walks them."""
    import ctypes as C
    abi = vio.abi
    n = 3
    keep = [np.eye(4, dtype=np.float32).reshape(16), np.eye(4, dtype=np.float32).reshape(16),
            np.arange(n, dtype=np.int32), np.tile(np.array([0, 0, 1], np.float32), n), np.ones(n, np.uint8),
            np.full(n, -1, np.int32), np.zeros(2 * n, np.float32),
            np.array([0, 2, 1, 3], np.int32), np.zeros(3, np.int32), np.zeros(3, np.int32)]
    f = abi.VioWindowFrame()
    f.frame_id, f.num_features, f.width = 5, n, 960
    f.T_wb, f.T_bc = abi._ptr(keep[0], C.c_float), abi._ptr(keep[1], C.c_float)
    f.feature_id, f.bearing = abi._ptr(keep[2], C.c_int32), abi._ptr(keep[3], C.c_float)
    f.valid, f.mappoint, f.uv = abi._ptr(keep[4], C.c_uint8), abi._ptr(keep[5], C.c_int32), abi._ptr(keep[6], C.c_float)
    f.track_begin, f.track_frame, f.track_feat = (abi._ptr(keep[7], C.c_int32), abi._ptr(keep[8], C.c_int32),
                                                  abi._ptr(keep[9], C.c_int32))
    w = vio.Window(10)
    st = abi.VioWindowKfStats()
    assert vio.lib().vio_window_add_keyframe(w.h, C.byref(f), C.byref(st)) == -22  # 2 > 1: not monotonic
    keep[7][:] = [0, 1, 2, 3]
    assert vio.lib().vio_window_add_keyframe(w.h, C.byref(f), C.byref(st)) == 0
    w.close()
