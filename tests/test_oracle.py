"""CPU tests of the oracle (oracle/ba_oracle.c): pinned by the Ceres known-answer tests the
reference ships (thirdparty/ceres-solver/internal/ceres/*_test.cc, restated here because they
cannot be compiled without Eigen) and by the independent numpy golden vectors in tests/golden/."""
import ctypes as C
import math
import os

import numpy as np
import pytest

import oracle_lib

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
dp = C.POINTER(C.c_double)


def _d(a):
    a = np.ascontiguousarray(a, np.float64)
    return a, a.ctypes.data_as(dp)


def test_lm_radius_schedule_kat():
    """levenberg_marquardt_strategy_test.cc:81-111 (AcceptRejectStepRadiusScaling)."""
    L = oracle_lib.load()
    q = np.array([0.0, -1.0, 1.0, 1.0, 0.25, 1.0, 1.0, 1.0])
    radii = np.zeros(len(q))
    L.oracle_lm_radius_schedule(C.c_double(2.0), C.c_double(20.0), _d(q)[1], len(q), radii.ctypes.data_as(dp))
    exp = [1.0, 0.25, 0.25 * 3, 0.25 * 9, 0.25 * 9 / 1.125, 0.25 * 9 / 1.125 * 3, 0.25 * 9 / 1.125 * 9, 20.0]
    assert radii.tolist() == exp  # EXPECT_EQ: exact


def test_lm_diagonal_kat():
    """levenberg_marquardt_strategy_test.cc:113-166: D = sqrt(clamp(diag)/radius)."""
    L = oracle_lib.load()
    L.oracle_lm_diagonal.argtypes = [C.c_int, dp, dp, C.c_double, C.c_double, C.c_double, dp]
    # J = [[0,1,100],[0,1,0]] -> diag(J^T J) = [0, 2, 10000], no scaling
    colsq, s, D = np.array([0.0, 2.0, 1e4]), np.ones(3), np.zeros(3)
    L.oracle_lm_diagonal(3, _d(colsq)[1], _d(s)[1], 2.0, 1e-2, 1e2, D.ctypes.data_as(dp))
    assert np.allclose(D, np.sqrt(np.array([1e-2, 2.0, 1e2]) / 2.0), rtol=0, atol=1e-15)


@pytest.mark.parametrize("delta", [0.7, 1.3])
@pytest.mark.parametrize("s", [0.357, 1.792])
def test_huber_kat(delta, s):
    """loss_function_test.cc:92-103 (AssertLossFunctionIsValid for HuberLoss)."""
    L = oracle_lib.load()
    L.oracle_huber.argtypes = [C.c_double, C.c_double, dp]

    def ev(x):
        r = np.zeros(3)
        L.oracle_huber(delta, x, r.ctypes.data_as(dp))
        return r

    rho, fwd, bwd, h = ev(s), ev(s + 1e-4), ev(s - 1e-4), 1e-4
    assert abs((fwd[0] - bwd[0]) / (2 * h) - rho[1]) < 1e-6
    assert abs((fwd[0] - 2 * rho[0] + bwd[0]) / (h * h) - rho[2]) < 1e-6
    assert np.allclose(ev(0.0), [0, 1, 0], atol=1e-6)


def test_corrector_scalar_kat():
    """corrector_test.cc:57-83: rho''<0 -> alpha = 0, scale sqrt(rho')."""
    L = oracle_lib.load()
    L.oracle_corrector.argtypes = [C.c_double, dp, dp, dp, dp]
    r, j = math.sqrt(3.0), 10.0
    rho = np.array([3.0, 0.1, -0.01])
    rs, asq, sr1 = C.c_double(), C.c_double(), C.c_double()
    L.oracle_corrector(3.0, rho.ctypes.data_as(dp), C.byref(rs), C.byref(asq), C.byref(sr1))
    assert abs(r * rs.value - r * math.sqrt(0.1)) < 1e-6
    assert asq.value == 0.0 and abs(sr1.value * j - math.sqrt(0.1) * j) < 1e-6


MASKS = [(1, 1, 1, 1), (1, 1, 1, 0), (1, 0, 1, 1), (0, 1, 1, 1), (1, 1, 0, 0), (1, 0, 1, 0), (0, 1, 1, 0),
         (1, 0, 0, 1), (0, 1, 0, 1), (0, 0, 1, 1), (1, 0, 0, 0), (0, 1, 0, 0), (0, 0, 1, 0), (0, 0, 0, 1)]


@pytest.mark.parametrize("mask", MASKS)
def test_powell_lm_kat(mask):
    """trust_region_minimizer_test.cc:224-294: LM on Powell's singular function reaches 0 +- 1e-3
    from (3,-1,0,1) for the 14 column masks the Ceres test runs."""
    L = oracle_lib.load()
    m = (C.c_int * 4)(*mask)
    x = np.array([3.0, -1.0, 0.0, 1.0]) * np.array(mask)
    it, fc, term = C.c_int(), C.c_double(), C.c_int()
    L.oracle_powell(m, x.ctypes.data_as(dp), C.byref(it), C.byref(fc), C.byref(term))
    assert np.all(np.abs(x) < 1e-3), (mask, x)


def test_nearest_rotation_matches_svd():
    """oracle_nearest_rotation == SO3d(Matrix3d) SVD projection (LieUtils.cpp:275-288)."""
    L = oracle_lib.load()
    rng = np.random.default_rng(0)
    for _ in range(200):
        A = rng.normal(size=(3, 3))
        if rng.random() < 0.5:  # near-orthonormal (f32-rounded rotation) like every input pose
            q, _ = np.linalg.qr(A)
            A = (q * np.sign(np.linalg.det(q))).astype(np.float32).astype(np.float64)
        U, _, Vt = np.linalg.svd(A)
        R = U @ Vt
        if np.linalg.det(R) < 0:
            U[:, 2] *= -1
            R = U @ Vt
        out = np.zeros(9)
        L.oracle_nearest_rotation(_d(A.reshape(-1))[1], out.ctypes.data_as(dp))
        assert np.abs(out.reshape(3, 3) - R).max() < 1e-12


def _pose(vio, T):
    return vio.abi.poses_to_c(T[None])


def test_factor_golden(vio):
    """C oracle BAFactor/PnPFactor vs the independent numpy golden vectors (rel 1e-12)."""
    L = oracle_lib.load()
    g = np.load(os.path.join(GOLDEN, "factor_golden.npz"))
    Tcb = _pose(vio, g["T_cb"])
    L.oracle_ba_chi2.restype = C.c_double
    n = len(g["ok"])
    branches = set()
    for i in range(n):
        T = _pose(vio, g["T"][i])
        r, Jp, Jl = np.zeros(2), np.zeros(12), np.zeros(6)
        delta, Pw = _d(g["delta"][i]), _d(g["Pw"][i])
        ok = L.oracle_ba_factor(T, Tcb, delta[1], Pw[1], C.c_double(g["obs"][i][0]), C.c_double(g["obs"][i][1]),
                                C.c_double(float(g["cols"])), C.c_double(float(g["rows"])), int(g["outlier"][i]),
                                int(g["is_pnp"][i]), r.ctypes.data_as(dp), Jp.ctypes.data_as(dp), Jl.ctypes.data_as(dp))
        assert bool(ok) == bool(g["ok"][i])
        if not ok:
            branches.add("pnp-fail")
            continue
        scale = 1.0 + np.abs(g["r"][i]).max()
        # x^2+z^2 < 1e-10 (landmark ~above the camera): atan2 of ~1e-6 m components amplifies the
        # 1e-16 rounding of Pc to ~1e-8 px, so that branch is compared at 1e-5 px
        degenerate = not np.any(g["Jp"][i]) and tuple(g["r"][i]) not in ((640.0, 480.0), (640.0, 360.0), (100.0, 100.0))
        tol = 1e-5 if degenerate else 1e-10 * scale
        assert np.abs(r - g["r"][i]).max() <= tol, (i, r, g["r"][i])
        js = 1.0 + np.abs(g["Jp"][i]).max()
        assert np.abs(Jp - g["Jp"][i].reshape(-1)).max() <= 1e-11 * js, i
        assert np.abs(Jl - g["Jl"][i].reshape(-1)).max() <= 1e-11 * js, i
        c2 = L.oracle_ba_chi2(T, Tcb, delta[1], Pw[1], C.c_double(g["obs"][i][0]), C.c_double(g["obs"][i][1]),
                              C.c_double(float(g["cols"])), C.c_double(float(g["rows"])), int(g["outlier"][i]),
                              int(g["is_pnp"][i]))
        ref = g["chi2"][i]
        assert abs(c2 - ref) <= (1e-3 if degenerate else 1e-9) * (1 + abs(ref)), (i, c2, ref)
        if tuple(g["r"][i]) in ((640.0, 480.0), (640.0, 360.0), (100.0, 100.0)):
            branches.add(tuple(g["r"][i]))
        elif not np.any(g["Jp"][i]):
            branches.add("jzero")
    # every special branch of Factors.cpp:331-476 is exercised
    assert {(640.0, 480.0), (640.0, 360.0), (100.0, 100.0), "jzero", "pnp-fail"} <= branches


def test_factor_jacobian_finite_difference(vio):
    """J_point is the true derivative; J_pose is the right-perturbation derivative at delta = 0
    (Factors.cpp:500-534) — check both by central differences."""
    L = oracle_lib.load()
    g = np.load(os.path.join(GOLDEN, "factor_golden.npz"))
    Tcb = _pose(vio, g["T_cb"])
    checked = 0
    for i in range(len(g["ok"])):
        if g["outlier"][i] or g["is_pnp"][i] or not np.any(g["Jp"][i]):
            continue
        T = _pose(vio, g["T"][i])
        obs = g["obs"][i]

        def res(delta, Pw):
            r = np.zeros(2)
            L.oracle_ba_factor(T, Tcb, _d(delta)[1], _d(Pw)[1], C.c_double(obs[0]), C.c_double(obs[1]),
                               C.c_double(960.0), C.c_double(480.0), 0, 0, r.ctypes.data_as(dp), None, None)
            return r

        d0, P0 = np.zeros(6), g["Pw"][i]
        Jp, Jl, r0 = np.zeros(12), np.zeros(6), np.zeros(2)
        L.oracle_ba_factor(T, Tcb, _d(d0)[1], _d(P0)[1], C.c_double(obs[0]), C.c_double(obs[1]), C.c_double(960.0),
                           C.c_double(480.0), 0, 0, r0.ctypes.data_as(dp), Jp.ctypes.data_as(dp),
                           Jl.ctypes.data_as(dp))
        if np.abs(r0).max() > 90:
            continue
        h = 1e-6
        for j in range(6):
            e = np.zeros(6); e[j] = h
            fd = (res(d0 + e, P0) - res(d0 - e, P0)) / (2 * h)
            assert np.allclose(fd, Jp.reshape(2, 6)[:, j], rtol=1e-4, atol=1e-3), (i, j)
        for j in range(3):
            e = np.zeros(3); e[j] = h
            fd = (res(d0, P0 + e) - res(d0, P0 - e)) / (2 * h)
            assert np.allclose(fd, Jl.reshape(2, 3)[:, j], rtol=1e-4, atol=1e-3), (i, j)
        checked += 1
    assert checked >= 20


@pytest.mark.parametrize("kw", [{}, dict(max_iterations=12, fixed_iterations=1)])
def test_oracle_trace_is_ceres_summary(vio, synth, kw):
    """Summary::iterations of the oracle obey Ceres' bookkeeping (trust_region_minimizer.cc): one
    entry per iteration incl. 0, iteration 0 valid + successful at initial_cost, final_cost = the
    smallest entry cost, the radius follows LevenbergMarquardtStrategy (accept: /max(1/3, 1-(2rho-1)^3),
    reject / invalid: /2, /4, ...), and an unsuccessful entry keeps the previous gradient norm."""
    import oracle_lib
    p = vio.BaProblem(synth.config3(), variant=vio.VIO_BA_VI, **kw)
    o = oracle_lib.ba_solve(vio, p)
    t = o["trace"]
    n = o["iterations"]
    assert len(t["cost"]) == n > 3
    assert list(t["iteration"]) == list(range(n))
    assert t["step_is_valid"][0] == t["step_is_successful"][0] == 1 and t["cost"][0] == o["initial_cost"]
    assert o["final_cost"] == t["cost"].min()
    assert t["trust_region_radius"][0] == 1e4
    dec = 2.0
    for i in range(1, n):
        r0, r1 = t["trust_region_radius"][i - 1], t["trust_region_radius"][i]
        if t["step_is_successful"][i]:
            q = t["relative_decrease"][i]
            assert q > 1e-3 and r1 == min(1e16, r0 / max(1 / 3, 1 - (2 * q - 1) ** 3))
            dec = 2.0
        else:
            assert r1 == r0 / dec and t["gradient_max_norm"][i] == t["gradient_max_norm"][i - 1]
            dec *= 2.0
        if t["step_is_valid"][i]:
            assert t["model_cost_change"][i] > 0


def test_config4_fixture_reproduces(vio, synth):
    """tests/golden/config4_oracle.json (the GPU config-4 test's reference) is this oracle's output."""
    import json
    import oracle_lib
    ref = json.load(open(os.path.join(GOLDEN, "config4_oracle.json")))["windows"]
    assert len(ref) == 256
    for i in (1, 3):
        o = oracle_lib.ba_solve(vio, vio.BaProblem(synth.config3(synth.SEED + i), variant=vio.VIO_BA_VI))
        assert o["iterations"] == ref[i]["iterations"] and o["final_cost"] == ref[i]["final_cost"]
        assert o["initial_cost"] == ref[i]["initial_cost"]


def test_config3_cloud_fixture_reproduces(vio, synth):
    """tests/golden/config3_cloud.json (the converged config-3 GPU bar) is this oracle's cloud: the
    unperturbed solve and two members regenerate exactly, and the cloud is wider than SURVEY §8c's
    bar where the GPU test widens it (so the widening is the reference's own sensitivity)."""
    import json
    import oracle_lib
    ref = json.load(open(os.path.join(GOLDEN, "config3_cloud.json")))
    w = synth.config3()
    o = oracle_lib.ba_solve(vio, vio.BaProblem(w, variant=vio.VIO_BA_VI))
    assert o["iterations"] == ref["oracle"]["iterations"] and o["final_cost"] == ref["oracle"]["final_cost"]
    for m in (ref["members"][1], ref["members"][4]):
        c = oracle_lib.ba_solve(vio, vio.BaProblem(dict(w, lm_xyz=w["lm_xyz"] * (1 + m["e"])), variant=vio.VIO_BA_VI))
        assert c["iterations"] == m["iterations"]
        assert np.abs(o["T_wb"][:, :3, 3] - c["T_wb"][:, :3, 3]).max() == m["pos_m"]
        assert np.abs(o["bg"] - c["bg"]).max() == m["bg"]
    mx = ref["max"]
    assert mx["pos_m"] > 1e-4 and mx["lm_m"] > 1e-3 and mx["bg"] > 1e-4 and mx["cost_rel"] > 1e-6
    assert ref["iterations_range"][1] - ref["iterations_range"][0] > 2


# ---- Schur complement: the reference's own Ceres fixtures -----------------------------------------
class OracleBsm(C.Structure):
    """oracle_bsm (oracle/ba_oracle.c): block-sparse matrix of the generic Schur eliminator."""
    _fields_ = [("n_cols", C.c_int), ("col_size", C.c_void_p), ("col_pos", C.c_void_p), ("col_red", C.c_void_p),
                ("n_red", C.c_int), ("n_rows", C.c_int), ("row_size", C.c_void_p), ("row_pos", C.c_void_p),
                ("row_cell", C.c_void_p), ("cell_col", C.c_void_p), ("cell_off", C.c_void_p), ("values", C.c_void_p)]


def bsm_from_fixture(pr):
    """The Ceres block structure (e-blocks first, CompressedRowBlockStructure) as an oracle_bsm plus
    its dense matrix."""
    cs = pr["col_sizes"]
    ne = pr["num_eliminate_blocks"]
    col_pos = np.cumsum([0] + cs[:-1]).astype(np.int32)
    ne_cols = int(sum(cs[:ne]))
    col_red = np.array([-1 if b < ne else int(col_pos[b]) - ne_cols for b in range(len(cs))], np.int32)
    row_size, row_pos, row_cell, cell_col, cell_off, vals = [], [], [0], [], [], []
    r0 = 0
    for rs, cells in pr["rows"]:
        row_size.append(rs)
        row_pos.append(r0)
        for cb, v in cells:
            assert len(v) == rs * cs[cb]
            cell_col.append(cb)
            cell_off.append(len(vals))
            vals.extend(v)
        row_cell.append(len(cell_col))
        r0 += rs
    dense = np.zeros((r0, int(sum(cs))))
    for r, (rs, cells) in enumerate(pr["rows"]):
        for cb, v in cells:
            dense[row_pos[r]:row_pos[r] + rs, col_pos[cb]:col_pos[cb] + cs[cb]] = np.array(v, float).reshape(rs, cs[cb])
    arrs = dict(col_size=np.array(cs, np.int32), col_pos=col_pos, col_red=col_red, row_size=np.array(row_size, np.int32),
                row_pos=np.array(row_pos, np.int32), row_cell=np.array(row_cell, np.int32),
                cell_col=np.array(cell_col, np.int32), cell_off=np.array(cell_off, np.int32),
                values=np.array(vals, np.float64))
    m = OracleBsm(len(cs), *[arrs[k].ctypes.data for k in ("col_size", "col_pos", "col_red")], int(sum(cs)) - ne_cols,
                  len(row_size), *[arrs[k].ctypes.data for k in ("row_size", "row_pos", "row_cell", "cell_col",
                                                                 "cell_off", "values")])
    return m, arrs, dense, ne_cols


def ceres_fixture(name):
    import json
    return json.load(open(os.path.join(GOLDEN, "ceres_lls_problems.json")))[name]


@pytest.mark.parametrize("name,reg", [("problem2", False), ("problem2", True), ("problem4", True)])
def test_schur_eliminator_ceres_kat(name, reg):
    """SchurEliminatorTest (schur_eliminator_test.cc:196-225: ScalarProblemNoRegularization,
    ScalarProblemWithRegularization, VaryingFBlockSize): the reduced system lhs / rhs and the
    back-substituted solution against the dense computation of ComputeReferenceSolution (:81-115),
    relative tolerance 1e-14, on LinearLeastSquaresProblem2 / 4 (tests/golden/ceres_lls_problems.json)."""
    L = oracle_lib.load()
    pr = ceres_fixture(name)
    A, keep, J, ne = bsm_from_fixture(pr)
    b = np.array(pr["b"], np.float64)
    D = np.array(pr["D"], np.float64) if reg else np.zeros(J.shape[1])
    # ComputeReferenceSolution: H = D^2 + J^T J, P = blockwise inverse of the e-e part
    H = np.diag(D * D) + J.T @ J
    g = J.T @ b
    P = H[:ne, :ne].copy()
    pos = 0
    for cb in range(pr["num_eliminate_blocks"]):
        sz = pr["col_sizes"][cb]
        P[pos:pos + sz, pos:pos + sz] = np.linalg.inv(P[pos:pos + sz, pos:pos + sz])
        pos += sz
    Q, R = H[:ne, ne:], H[ne:, ne:]
    lhs_e = R - Q.T @ P @ Q
    rhs_e = g[ne:] - Q.T @ P @ g[:ne]
    sol_e = np.linalg.solve(H, g)
    S = J.shape[1] - ne
    lhs, rhs, x = np.zeros((S, S)), np.zeros(S), np.zeros(J.shape[1])
    L.oracle_schur_eliminate.argtypes = [C.POINTER(OracleBsm), dp, dp, dp, dp]
    L.oracle_schur_solve.argtypes = [C.POINTER(OracleBsm), dp, dp, dp]
    assert L.oracle_schur_eliminate(C.byref(A), _d(b)[1], _d(D)[1], lhs.ctypes.data_as(dp), rhs.ctypes.data_as(dp)) == 1
    assert L.oracle_schur_solve(C.byref(A), _d(b)[1], _d(D)[1], x.ctypes.data_as(dp)) == 1
    assert np.linalg.norm(np.triu(lhs - lhs_e)) / np.linalg.norm(lhs_e) <= 1e-14
    assert np.linalg.norm(rhs - rhs_e) / np.linalg.norm(rhs_e) <= 1e-14
    assert np.linalg.norm(x - sol_e) / np.linalg.norm(sol_e) <= 1e-14


@pytest.mark.parametrize("name,reg", [("problem2", False), ("problem2", True), ("problem3", False),
                                      ("problem3", True), ("problem4", True)])
def test_schur_complement_solver_ceres_kat(name, reg):
    """SchurComplementSolverTest (schur_complement_solver_test.cc:50-220, DENSE_SCHUR / SPARSE_SCHUR on
    problems 2, 3 — every column eliminated — and 4): |x - x_QR| / num_cols <= 1e-10 against the dense
    least-squares solution of [A; diag(D)] x = [b; 0]."""
    L = oracle_lib.load()
    pr = ceres_fixture(name)
    A, keep, J, ne = bsm_from_fixture(pr)
    b = np.array(pr["b"], np.float64)
    n = J.shape[1]
    D = np.array(pr["D"], np.float64) if reg else None
    Aa = np.vstack([J, np.diag(D)]) if reg else J
    ba = np.concatenate([b, np.zeros(n)]) if reg else b
    x_qr = np.linalg.lstsq(Aa, ba, rcond=None)[0]
    x = np.zeros(n)
    L.oracle_schur_solve.argtypes = [C.POINTER(OracleBsm), dp, dp, dp]
    assert L.oracle_schur_solve(C.byref(A), _d(b)[1], _d(D)[1] if reg else None, x.ctypes.data_as(dp)) == 1
    assert np.linalg.norm(x - x_qr) / n <= 1e-10


def test_jacobi_scaling_ceres_kat():
    """JacobiScalingTest (trust_region_minimizer_test.cc:389-410): a closed 6-vertex polygon on the unit
    circle stretched to perimeter 10 through one residual, LM + DENSE_QR with Jacobi scaling (the
    default options): final_cost <= 1e-10."""
    L = oracle_lib.load()
    N = 6
    th = np.arange(N) * 2.0 * 3.1415926535897932384626433 / N
    y = np.stack([np.cos(th), np.sin(th)], 1).reshape(-1).copy()
    fc, it, term = C.c_double(), C.c_int(), C.c_int()
    L.oracle_curve_kat.argtypes = [C.c_int, C.c_double, dp, C.POINTER(C.c_double), C.POINTER(C.c_int),
                                   C.POINTER(C.c_int)]
    assert L.oracle_curve_kat(N, 10.0, y.ctypes.data_as(dp), C.byref(fc), C.byref(it), C.byref(term)) == 0
    assert fc.value <= 1e-10
    per = sum(np.linalg.norm(y.reshape(N, 2)[i] - y.reshape(N, 2)[i - 1]) for i in range(N))
    assert abs(per - 10.0) <= 1e-4


def test_threaded_baseline_legs(vio, synth):
    """The CPU-baseline leg's threaded oracle (oracle_set_threads > 1): the tracker loops are per-pixel
    / per-point independent, so 4 threads are bitwise the 1-thread result; the BA solve reorders its
    sums (Schur partials per thread), so it agrees to roundoff amplification only."""
    L = oracle_lib.load()
    a, b, _ = synth.config1(640, 320)
    H, W = a.shape
    mask = np.full((H, W), 255, np.uint8)
    kp = vio.default_klt_params()
    try:
        outs = []
        for T in (1, 4):
            L.oracle_set_threads(T)
            pts = oracle_lib.gftt(a, mask, 200, float(np.float32(0.01)), 10.0)
            nxt, st, err = oracle_lib.klt_track(a, b, pts, kp)
            outs.append((pts, nxt, st, err, oracle_lib.min_eig_map(b), oracle_lib.pyr_down(b)))
        for x, y in zip(*outs):
            np.testing.assert_array_equal(x, y)
        p = vio.BaProblem(synth.config3(), variant=vio.VIO_BA_VI, max_iterations=5, fixed_iterations=1)
        res = []
        for T in (1, 4):
            L.oracle_set_threads(T)
            res.append(oracle_lib.ba_solve(vio, p))
        assert res[0]["iterations"] == res[1]["iterations"]
        assert abs(res[0]["final_cost"] - res[1]["final_cost"]) <= 1e-9 * res[0]["final_cost"]
        np.testing.assert_allclose(res[0]["lm_xyz"], res[1]["lm_xyz"], rtol=0, atol=1e-6)
    finally:
        L.oracle_set_threads(1)
