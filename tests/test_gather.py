"""Problem assembly (a4) and write-back (a3 host half): libvio360's vio_ba_gather / vio_ba_write_back
against a Python restatement of the Optimizer entry points' rules, on random Frame / Feature /
MapPoint graphs with every filter exercised (invalid features, null and bad MapPoints, near-boundary
pixels, marginalised MapPoints, observations of frames outside the window, frames without a
residual, too few frames / MapPoints / PnP observations).

Restated from /root/reference/src/optimization/Optimizer.cpp:
  SolvePnP :83-130, :272-297   RunBA :303-409, :459-474   RunVIBA :493-636, :684-712
  RunLocalBA :726-851, :917-954   IsNearBoundary :41-46 -> Camera.cpp:134-139
The reference orders MapPoints by std::set<shared_ptr> (pointer order); the view's mp_key stands in.
"""
import numpy as np
import pytest

LOCAL, FULL, VI, PNP = 0, 1, 2, 3


# ------------------------------------------------------------------------------------------------
# Python restatement
def near_boundary(uv, W, H, margin):
    """Camera::IsNearBoundary in f32 (margin <= 0: Optimizer::IsNearBoundary returns false)."""
    if margin <= 0:
        return False
    m, x, y = np.float32(margin), np.float32(uv[0]), np.float32(uv[1])
    return bool(x < m or x > np.float32(W) - m or y < m or y > np.float32(H) - m)


def ref_gather(G, variant, fix_first, fix_last):
    fb, fmp, fvalid = G["feat_begin"], G["feat_mp"], G["feat_valid"]
    F = len(fb) - 1
    W, H, mg = G["width"], G["height"], G["boundary_margin"]
    nb = lambda g: near_boundary(G["feat_uv"][g], W, H, mg)  # noqa: E731

    def usable(g):  # `feature && feature->IsValid()`, `mp && !mp->IsBad()`
        return bool(fvalid[g]) and fmp[g] >= 0 and not G["mp_bad"][fmp[g]]

    out = {"status": 0, "lm_mp": [], "lm_const": [], "obs": [], "kf_const": np.zeros(F, np.uint8),
           "kf_in_problem": np.zeros(F, np.uint8)}
    if variant == PNP:
        obs = [g for g in range(fb[0], fb[1]) if usable(g) and not nb(g)] if F >= 1 else []
        if len(obs) < 6:
            out["status"] = 3
            return out
        for g in obs:
            out["lm_mp"].append(fmp[g])
            out["lm_const"].append(G["mp_marg"][fmp[g]])
            out["obs"].append((0, len(out["lm_mp"]) - 1, g))
        out["kf_in_problem"][0] = 1
        return out
    if F < 2:
        out["status"] = 1
        return out
    mappoint_set = {fmp[g] for g in range(fb[F]) if usable(g)}
    mappoints = sorted(mappoint_set, key=lambda m: G["mp_key"][m])
    if not mappoints:
        out["status"] = 2
        return out
    mp_to_idx = {mp: i for i, mp in enumerate(mappoints)}
    out["lm_mp"] = mappoints
    if variant == LOCAL:
        for pi, mp in enumerate(mappoints):
            for q in range(G["mp_obs_begin"][mp], G["mp_obs_begin"][mp + 1]):
                f, fi = G["mp_obs_frame"][q], G["mp_obs_feat"][q]
                if f < 0:  # expired frame / frame_to_idx.find == end
                    continue
                if fi < 0 or fi >= fb[f + 1] - fb[f]:
                    continue
                g = fb[f] + fi
                if not fvalid[g] or nb(g):
                    continue
                out["obs"].append((f, pi, g))
        poses_in_problem = {f for f, _, _ in out["obs"]}
        for f in poses_in_problem:
            out["kf_in_problem"][f] = 1
        if 0 in poses_in_problem:  # NUM_FIXED_KEYFRAMES = 1
            out["kf_const"][0] = 1
        out["lm_const"] = [G["mp_marg"][m] for m in mappoints]
        return out
    for f in range(F):
        for g in range(fb[f], fb[f + 1]):
            if not usable(g) or nb(g):
                continue
            if fmp[g] not in mp_to_idx:
                continue
            out["obs"].append((f, mp_to_idx[fmp[g]], g))
            out["kf_in_problem"][f] = 1
    if fix_first:
        out["kf_const"][0] = 1
    if variant == FULL and fix_last and F > 1:
        out["kf_const"][F - 1] = 1
    out["lm_const"] = [0] * len(mappoints)
    return out


def f32_pose(T):
    M = np.zeros((4, 4), np.float32)
    M[:3, :4] = np.asarray(T, np.float64)[:3, :4].astype(np.float32)
    M[3, 3] = 1.0
    return M


def ref_write_back(G, variant, ref_g, res):
    F, M = len(G["feat_begin"]) - 1, len(G["mp_key"])
    u = {"frame_set": np.zeros(F, np.uint8), "frame_Twb": {}, "mp_set": np.zeros(M, np.uint8), "mp_pos": {},
         "mp_set_bad": np.zeros(M, np.uint8), "success": 0, "num_poses_optimized": 0, "num_points_optimized": 0}
    if ref_g["status"] != 0:
        return u
    u["success"] = res["success"]
    if variant == PNP:
        if res["num_inliers"] >= 10:
            u["frame_set"][0] = 1
            u["frame_Twb"][0] = f32_pose(res["T_wb"][0])
        return u
    for l, mp in enumerate(ref_g["lm_mp"]):
        if res["lm_bad"][l]:
            u["mp_set_bad"][mp] = 1
    u["num_points_optimized"] = len(ref_g["lm_mp"])
    if variant == LOCAL:
        for f in range(1, F):
            if ref_g["kf_in_problem"][f]:
                u["frame_set"][f] = 1
                u["frame_Twb"][f] = f32_pose(res["T_wb"][f])
        u["num_poses_optimized"] = F - 1 + int(ref_g["kf_in_problem"][0])
        for l, mp in enumerate(ref_g["lm_mp"]):
            if not G["mp_marg"][mp]:
                u["mp_set"][mp] = 1
                u["mp_pos"][mp] = res["lm_xyz"][l].astype(np.float32)
        return u
    for f in range(F):
        u["frame_set"][f] = 1
        u["frame_Twb"][f] = f32_pose(res["T_wb"][f])
    u["num_poses_optimized"] = F
    for l, mp in enumerate(ref_g["lm_mp"]):
        if not res["lm_bad"][l] and not G["mp_marg"][mp]:
            u["mp_set"][mp] = 1
            u["mp_pos"][mp] = res["lm_xyz"][l].astype(np.float32)
    return u


# ------------------------------------------------------------------------------------------------
# random graphs
def random_graph(seed, F=6, M=60, W=960, H=480, margin=20):
    rng = np.random.default_rng(seed)
    feat_begin, feat_uv, feat_valid, feat_mp = [0], [], [], []
    for f in range(F):
        n = int(rng.integers(0, 40)) if f != 2 else 0  # frame 2 has no features at all
        for _ in range(n):
            u = rng.uniform(-5, W + 5) if rng.random() < 0.15 else rng.uniform(0, W)
            v = rng.uniform(-5, H + 5) if rng.random() < 0.15 else rng.uniform(0, H)
            if rng.random() < 0.05:
                u = margin  # exactly on the margin: not near (strict <)
            feat_uv.append((u, v))
            feat_valid.append(rng.random() > 0.1)
            feat_mp.append(int(rng.integers(0, M)) if rng.random() > 0.1 else -1)
        feat_begin.append(len(feat_uv))
    Gn = len(feat_uv)
    mp_obs = [[] for _ in range(M)]
    for f in range(F):
        for i in range(feat_begin[f + 1] - feat_begin[f]):
            mp = feat_mp[feat_begin[f] + i]
            if mp >= 0:
                mp_obs[mp].append((f, i))
    for mp in range(M):  # observations from frames outside the window / stale feature indices
        if rng.random() < 0.3:
            mp_obs[mp].insert(int(rng.integers(0, len(mp_obs[mp]) + 1)), (-1, int(rng.integers(0, 10))))
        if rng.random() < 0.1:
            mp_obs[mp].append((int(rng.integers(0, F)), 999))
    obs_begin = np.cumsum([0] + [len(o) for o in mp_obs]).astype(np.int32)
    Tw = np.tile(np.eye(4, dtype=np.float32), (F, 1, 1))
    Tw[:, :3, 3] = rng.normal(0, 1, (F, 3))
    return {
        "frame_Twb": Tw, "frame_Tcb": np.tile(np.eye(4, dtype=np.float32), (F, 1, 1)),
        "feat_begin": np.array(feat_begin, np.int32),
        "feat_uv": np.array(feat_uv, np.float32).reshape(Gn, 2),
        "feat_valid": np.array(feat_valid, np.uint8), "feat_mp": np.array(feat_mp, np.int32),
        "mp_key": rng.permutation(M * 7)[:M].astype(np.int64),
        "mp_bad": (rng.random(M) < 0.1).astype(np.uint8), "mp_marg": (rng.random(M) < 0.2).astype(np.uint8),
        "mp_pos": rng.normal(0, 5, (M, 3)).astype(np.float32),
        "mp_obs_begin": obs_begin,
        "mp_obs_frame": np.array([f for o in mp_obs for f, _ in o], np.int32),
        "mp_obs_feat": np.array([i for o in mp_obs for _, i in o], np.int32),
        "width": W, "height": H, "boundary_margin": margin,
    }


def assert_gather_equal(G, r, ref):
    assert r["status"] == ref["status"]
    if ref["status"]:
        return
    np.testing.assert_array_equal(r["lm_mp"], ref["lm_mp"])
    np.testing.assert_array_equal(r["lm_const"], np.asarray(ref["lm_const"], np.uint8))
    np.testing.assert_array_equal(r["lm_marg"], G["mp_marg"][r["lm_mp"]])
    np.testing.assert_array_equal(r["lm_xyz"], G["mp_pos"][r["lm_mp"]].astype(np.float64))
    obs = np.array(ref["obs"], np.int64).reshape(-1, 3)
    np.testing.assert_array_equal(r["obs_kf"], obs[:, 0])
    np.testing.assert_array_equal(r["obs_lm"], obs[:, 1])
    np.testing.assert_array_equal(r["obs_feat"], obs[:, 2])
    np.testing.assert_array_equal(r["obs_uv"], G["feat_uv"][obs[:, 2]])
    np.testing.assert_array_equal(r["kf_const"], ref["kf_const"])
    np.testing.assert_array_equal(r["kf_in_problem"], ref["kf_in_problem"])
    np.testing.assert_array_equal(r["T_wb_init"][:, :3, :], G["frame_Twb"][:, :3, :].astype(np.float64))


CASES = [(LOCAL, 1, 0), (FULL, 1, 0), (FULL, 1, 1), (FULL, 0, 0), (VI, 1, 0), (VI, 0, 0), (PNP, 0, 0)]


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("variant,fix_first,fix_last", CASES)
def test_gather_matches_restatement(vio, seed, variant, fix_first, fix_last):
    G = random_graph(seed)
    view = vio.abi.MapView(G)
    g = vio.ba_gather(view, variant, fix_first, fix_last)
    assert_gather_equal(G, g.result(), ref_gather(G, variant, fix_first, fix_last))


def _fake_output(vio, g, K, seed):
    """A solver output with arbitrary values (the write-back only routes them)."""
    rng = np.random.default_rng(seed)
    L, N = g.c.num_lm, g.c.num_obs
    O = vio.BaOutput(K, max(L, 1), max(N, 1))
    for k in range(K):
        O.T_wb[k].R[:] = rng.normal(0, 1, 9).tolist()
        O.T_wb[k].t[:] = rng.normal(0, 1, 3).tolist()
    O.lm_xyz[:] = rng.normal(0, 3, O.lm_xyz.shape)
    O.lm_bad[:] = (rng.random(O.lm_bad.shape) < 0.3).astype(np.uint8)
    O.vel[:] = rng.normal(0, 1, O.vel.shape)
    O.bg[:], O.ba[:] = rng.normal(0, 1, 3), rng.normal(0, 1, 3)
    s = O.summary
    s.success, s.num_inliers, s.num_outliers, s.iterations = 1, int(rng.integers(0, 20)), 3, 7
    s.initial_cost, s.final_cost = 10.0, 2.0
    res = O.result()
    res["T_wb"] = np.array([[list(O.T_wb[k].R[0:3]) + [O.T_wb[k].t[0]], list(O.T_wb[k].R[3:6]) + [O.T_wb[k].t[1]],
                             list(O.T_wb[k].R[6:9]) + [O.T_wb[k].t[2]]] for k in range(K)])
    return O, res


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("variant,fix_first,fix_last", CASES)
def test_write_back_matches_restatement(vio, seed, variant, fix_first, fix_last):
    G = random_graph(100 + seed)
    view = vio.abi.MapView(G)
    g = vio.ba_gather(view, variant, fix_first, fix_last)
    ref_g = ref_gather(G, variant, fix_first, fix_last)
    F = view.F
    O, res = _fake_output(vio, g, F, seed)
    u = vio.ba_write_back(view, variant, g, O if g.c.status == 0 else None)
    ref = ref_write_back(G, variant, ref_g, res)
    np.testing.assert_array_equal(u["frame_set"], ref["frame_set"])
    for f, T in ref["frame_Twb"].items():
        np.testing.assert_array_equal(u["frame_Twb"][f], T)
    np.testing.assert_array_equal(u["mp_set"], ref["mp_set"])
    np.testing.assert_array_equal(u["mp_set_bad"], ref["mp_set_bad"])
    for mp, p in ref["mp_pos"].items():
        np.testing.assert_array_equal(u["mp_pos"][mp], p)
    assert u["success"] == ref["success"]
    assert u["num_poses_optimized"] == ref["num_poses_optimized"]
    assert u["num_points_optimized"] == ref["num_points_optimized"]
    if g.c.status == 0 and variant == VI:
        np.testing.assert_array_equal(u["frame_vel"], res["vel"].astype(np.float32))
        np.testing.assert_array_equal(u["bias"], np.concatenate([res["bg"], res["ba"]]).astype(np.float32))


def test_guard_statuses(vio):
    G = random_graph(5)
    one = {k: v for k, v in G.items()}
    one["feat_begin"] = G["feat_begin"][:2]
    one["frame_Twb"], one["frame_Tcb"] = G["frame_Twb"][:1], G["frame_Tcb"][:1]
    v1 = vio.abi.MapView(one)
    for variant in (LOCAL, FULL, VI):
        g = vio.ba_gather(v1, variant)
        assert g.c.status == vio.abi.VIO_GATHER_FEW_FRAMES
        u = vio.ba_write_back(v1, variant, g, None)
        assert u["success"] == 0 and not u["frame_set"].any() and not u["mp_set"].any()
    allbad = dict(G, mp_bad=np.ones_like(G["mp_bad"]))
    assert vio.ba_gather(vio.abi.MapView(allbad), FULL).c.status == vio.abi.VIO_GATHER_NO_MAPPOINTS
    assert vio.ba_gather(vio.abi.MapView(allbad), PNP).c.status == vio.abi.VIO_GATHER_FEW_OBS
    # margin <= 0 disables IsNearBoundary: every usable feature becomes a residual
    nomargin = dict(G, boundary_margin=0)
    r = vio.ba_gather(vio.abi.MapView(nomargin), FULL).result()
    assert_gather_equal(nomargin, r, ref_gather(nomargin, FULL, 1, 0))
    with pytest.raises(vio.VioError):  # MapPoint keys must be unique (std::set of distinct objects)
        vio.ba_gather(vio.abi.MapView(dict(G, mp_key=np.zeros_like(G["mp_key"]))), FULL)


def graph_from_window(w, seed=0, extra=True):
    """A Frame / Feature / MapPoint graph whose RunBA gather is the synthetic window `w` (plus filtered
    noise: invalid features, features without / with bad MapPoints, near-boundary features)."""
    rng = np.random.default_rng(seed)
    K, L = len(w["T_wb_init"]), len(w["lm_xyz"])
    feats = [[] for _ in range(K)]
    for o in range(len(w["obs_kf"])):
        feats[w["obs_kf"][o]].append((tuple(w["obs_uv"][o]), True, int(w["obs_lm"][o])))
    M = L + (5 if extra else 0)  # 5 bad MapPoints
    if extra:
        for k in range(K):
            for _ in range(4):
                uv = (float(rng.uniform(100, w["cols"] - 100)), float(rng.uniform(100, w["rows"] - 100)))
                kind = rng.integers(0, 3)
                feats[k].insert(int(rng.integers(0, len(feats[k]) + 1)),
                                (uv, kind != 0, -1 if kind == 1 else int(L + rng.integers(0, 5))))
            feats[k].append(((5.0, 200.0), True, int(rng.integers(0, L))))  # near the boundary
    feat_begin = np.cumsum([0] + [len(f) for f in feats]).astype(np.int32)
    flat = [x for f in feats for x in f]
    mp_obs = [[] for _ in range(M)]
    for k in range(K):
        for i, (_, _, mp) in enumerate(feats[k]):
            if mp >= 0:
                mp_obs[mp].append((k, i))
    Tw = np.tile(np.eye(4, dtype=np.float32), (K, 1, 1))
    Tw[:, :3, :] = np.asarray(w["T_wb_init"])[:, :3, :].astype(np.float32)
    Tcb = np.asarray(w["T_cb"], np.float32)
    return {
        "frame_Twb": Tw, "frame_Tcb": np.repeat(Tcb[None], K, 0) if Tcb.ndim == 2 else Tcb,
        "feat_begin": feat_begin, "feat_uv": np.array([x[0] for x in flat], np.float32),
        "feat_valid": np.array([x[1] for x in flat], np.uint8), "feat_mp": np.array([x[2] for x in flat], np.int32),
        "mp_key": np.arange(M, dtype=np.int64), "mp_bad": np.r_[np.zeros(L), np.ones(M - L)].astype(np.uint8),
        "mp_marg": np.r_[w.get("lm_marg", np.zeros(L)), np.zeros(M - L)].astype(np.uint8),
        "mp_pos": np.r_[np.asarray(w["lm_xyz"]), np.zeros((M - L, 3))].astype(np.float32),
        "mp_obs_begin": np.cumsum([0] + [len(o) for o in mp_obs]).astype(np.int32),
        "mp_obs_frame": np.array([k for o in mp_obs for k, _ in o], np.int32),
        "mp_obs_feat": np.array([i for o in mp_obs for _, i in o], np.int32),
        "width": int(w["cols"]), "height": int(w["rows"]), "boundary_margin": 20,
    }


def test_gather_reproduces_window_and_oracle_write_back(vio, synth):
    """End to end on the CPU leg: graph -> vio_ba_gather (RunBA) -> the oracle solve of the gathered
    problem -> vio_ba_write_back; the gathered problem is the synthetic window itself (frame-major
    order), and the written positions / poses are the f32 casts of the solution."""
    import oracle_lib
    w = synth.config2()
    G = graph_from_window(w)
    view = vio.abi.MapView(G)
    g = vio.ba_gather(view, FULL, True, False)
    r = g.result()
    assert r["status"] == 0
    order = np.lexsort((np.arange(len(w["obs_kf"])), w["obs_kf"]))  # RunBA: frame-major
    np.testing.assert_array_equal(r["obs_kf"], w["obs_kf"][order])
    np.testing.assert_array_equal(r["obs_lm"], w["obs_lm"][order])
    np.testing.assert_array_equal(r["obs_uv"], w["obs_uv"][order])
    np.testing.assert_array_equal(r["lm_mp"], np.arange(len(w["lm_xyz"])))
    p = vio.BaProblem(g.window(view), variant=FULL, max_iterations=10)
    O = vio.BaOutput(p.K, p.L, p.N)
    import ctypes as C
    assert oracle_lib.load().oracle_ba_solve(C.byref(p.c), C.byref(O.c)) == 0
    u = vio.ba_write_back(view, FULL, g, O)
    res = O.result()
    assert u["frame_set"].all() and u["num_poses_optimized"] == p.K
    np.testing.assert_array_equal(u["frame_Twb"][:, :3, :], res["T_wb"][:, :3, :].astype(np.float32))
    keep = ~res["lm_bad"].astype(bool)
    np.testing.assert_array_equal(u["mp_set"][: p.L], keep.astype(np.uint8))
    np.testing.assert_array_equal(u["mp_pos"][: p.L][keep], res["lm_xyz"][keep].astype(np.float32))
    assert not u["mp_set"][p.L:].any()


@pytest.mark.gpu
def test_gpu_solve_write_back_matches_oracle(vio, synth):
    """The HIP solve of a gathered RunLocalBA problem written back like the oracle's (positions to f32
    within the BA parity tolerance, identical SetBad / SetPosition / SetTwb sets)."""
    import ctypes as C
    import oracle_lib
    w = synth.config2()
    G = graph_from_window(w, seed=3)
    view = vio.abi.MapView(G)
    g = vio.ba_gather(view, LOCAL)
    p = vio.BaProblem(g.window(view), variant=LOCAL, max_iterations=10, fixed_iterations=1)
    ctx = vio.Context(0)
    try:
        Og = vio.BaOutput(p.K, p.L, p.N)
        ctx.check(vio.lib().vio_ba_solve(ctx.h, C.byref(p.c), C.byref(Og.c)), "vio_ba_solve")
    finally:
        ctx.close()
    Oo = vio.BaOutput(p.K, p.L, p.N)
    assert oracle_lib.load().oracle_ba_solve(C.byref(p.c), C.byref(Oo.c)) == 0
    ug, uo = vio.ba_write_back(view, LOCAL, g, Og), vio.ba_write_back(view, LOCAL, g, Oo)
    for k in ("frame_set", "mp_set", "mp_set_bad"):
        np.testing.assert_array_equal(ug[k], uo[k])
    np.testing.assert_allclose(ug["frame_Twb"], uo["frame_Twb"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(ug["mp_pos"], uo["mp_pos"], rtol=0, atol=1e-4)
