"""GPU parity of the HIP sliding-window BA (libvio360.so via the C-ABI) against the CPU oracle.

Tolerances (stated in SURVEY §8c and DESIGN.md): final poses |dt| <= 1e-4 m and rotation angle
<= 1e-5 rad, landmarks <= 1e-3 m, final cost rel 1e-6, iteration count +-1, outlier flags
identical except for observations whose chi^2 lies within 1e-6 (relative) of the threshold.
The HIP path reorders floating-point sums (fixed-order wave reductions instead of the oracle's
sequential loops), so results agree to roundoff, not bitwise; the HIP path itself IS bitwise
reproducible (no atomics) and is tested for that below.
"""
import math

import numpy as np
import pytest

import oracle_lib

pytestmark = pytest.mark.gpu


def rot_angle(Ra, Rb):
    c = (np.trace(Ra.T @ Rb) - 1.0) / 2.0
    return math.acos(max(-1.0, min(1.0, c)))


def assert_parity(o, g, thr, iters_tol=1, cost_rtol=1e-6):
    K = len(o["T_wb"])
    for k in range(K):
        assert np.abs(o["T_wb"][k, :3, 3] - g["T_wb"][k, :3, 3]).max() <= 1e-4, k
        assert rot_angle(o["T_wb"][k, :3, :3], g["T_wb"][k, :3, :3]) <= 1e-5, k
    if len(o["lm_xyz"]):
        assert np.abs(o["lm_xyz"] - g["lm_xyz"]).max() <= 1e-3
    assert abs(o["iterations"] - g["iterations"]) <= iters_tol, (o["iterations"], g["iterations"])
    assert o["termination"] == g["termination"] or abs(o["iterations"] - g["iterations"]) <= iters_tol
    assert o["success"] == g["success"]
    assert abs(o["initial_cost"] - g["initial_cost"]) <= 1e-9 * max(1.0, abs(o["initial_cost"]))
    assert abs(o["final_cost"] - g["final_cost"]) <= cost_rtol * max(1.0, abs(o["final_cost"]))
    near = np.abs(o["obs_chi2"] - thr) <= 1e-6 * thr
    assert np.array_equal(o["obs_outlier"][~near], g["obs_outlier"][~near])
    fin = np.isfinite(o["obs_chi2"]) & (o["obs_chi2"] < 1e300)
    assert np.allclose(o["obs_chi2"][fin], g["obs_chi2"][fin], rtol=1e-4, atol=1e-4)


def cases(vio, synth):
    return [
        ("cfg2-local", synth.config2(), vio.VIO_BA_LOCAL),
        ("cfg2-full", synth.config2(), vio.VIO_BA_FULL),
        ("cfg3-vi", synth.config3(), vio.VIO_BA_VI),
        ("local-marg-outliers", synth.make_window(K=8, L=150, seed=3, marg_frac=0.2, outlier_frac=0.05,
                                                  all_visible=False), vio.VIO_BA_LOCAL),
        ("full-outliers", synth.make_window(K=6, L=120, seed=11, outlier_frac=0.08, all_visible=False),
         vio.VIO_BA_FULL),
        ("vi-K6", synth.make_window(K=6, L=80, seed=5, imu=True), vio.VIO_BA_VI),
        ("pnp", synth.make_pnp(synth.config2(), outlier_frac=0.1, marg_frac=0.1), vio.VIO_PNP),
        ("pnp-clean", synth.make_pnp(synth.config2(), kf=4), vio.VIO_PNP),
    ]


@pytest.fixture(scope="module")
def all_cases(vio, synth):
    return cases(vio, synth)


# ---- LM trace parity (Solver::Summary::iterations, vio_ba_output.trace) ----------------------------
PERTURB = (1e-15, -1e-15, 1e-14, -1e-14)  # relative changes of the landmark inputs: 5-50 ulp


def oracle_cloud(vio, w, variant, **kw):
    """The oracle on the window and on copies whose landmark inputs moved by a few ulp: how far
    the reference algorithm itself moves under input roundoff (its numerical sensitivity)."""
    return [oracle_lib.ba_solve(vio, vio.BaProblem(dict(w, lm_xyz=w["lm_xyz"] * (1 + e)), variant=variant, **kw))
            for e in PERTURB]


def roundoff_decided(tr, i, fixed):
    """Is iteration i's accept / stop decision decided by roundoff?  Its margin in cost units —
    |cost_change - 1e-3 model_change| for the rho > 1e-3 test (trust_region_step_evaluator.cc),
    ||cost_change| - 1e-6 cost| for the function tolerance (trust_region_minimizer.cc:740-760) — is
    within 1e-11 of the cost, i.e. within the roundoff of a cost summed over thousands of terms."""
    if not tr["step_is_valid"][i] or i == 0:
        return False
    cost, dc, m = tr["cost"][i - 1], tr["cost_change"][i], tr["model_cost_change"][i]
    tol = 1e-11 * abs(cost)
    if abs(dc - 1e-3 * m) <= tol:
        return True
    return not fixed and abs(abs(dc) - 1e-6 * abs(cost)) <= tol


def compare_traces(o, g, cloud, fixed, min_prefix):
    """GPU vs oracle Summary::iterations up to the first roundoff-decided iteration (or the first
    where the perturbed oracles disagree on a decision): identical decisions and iteration numbers,
    and per-iteration costs within max(1e-12, 10 x the perturbed-oracle spread) relative.  Returns
    the compared prefix length."""
    to, tg = o["trace"], g["trace"]
    n = min(len(to["cost"]), len(tg["cost"]))
    stop = n
    for i in range(n):
        dis = any(i >= len(c["trace"]["cost"]) or c["trace"]["step_is_successful"][i] != to["step_is_successful"][i]
                  for c in cloud)
        if roundoff_decided(to, i, fixed) or dis:
            stop = i
            break
    assert stop >= min_prefix, (stop, min_prefix)
    for i in range(stop):
        assert tg["iteration"][i] == to["iteration"][i] == i
        assert tg["step_is_valid"][i] == to["step_is_valid"][i], i
        assert tg["step_is_successful"][i] == to["step_is_successful"][i], i
        env = max(abs(c["trace"]["cost"][i] - to["cost"][i]) for c in cloud) / to["cost"][i]
        rel = abs(tg["cost"][i] - to["cost"][i]) / to["cost"][i]
        assert rel <= max(1e-12, 10 * env), (i, rel, env)
        assert abs(tg["trust_region_radius"][i] - to["trust_region_radius"][i]) <= \
            max(1e-9, 10 * max(abs(c["trace"]["trust_region_radius"][i] - to["trust_region_radius"][i])
                               for c in cloud) / to["trust_region_radius"][i]) * to["trust_region_radius"][i], i
    return stop


TRACE_CASES = [  # (case index in cases(), solver kwargs, min compared prefix)
    (2, {}, 30),                                            # config 3, reference options (tolerance-terminated)
    (2, dict(max_iterations=30, fixed_iterations=1), 31),   # config 3, the timed fixed-iteration mode
    (5, dict(max_iterations=40, fixed_iterations=1), 20),   # VI K=6 far past convergence
    (0, {}, 5),                                             # config 2 LocalBA
    (3, {}, 5),                                             # LocalBA with marginalised MPs and outliers
]


@pytest.mark.parametrize("tc", range(len(TRACE_CASES)))
def test_lm_trace_matches_oracle(vio, gpu_ctx, all_cases, tc):
    """Per-iteration LM trace (cost, step validity / acceptance, radius) of both execution routes
    against the oracle's, up to the first decision that roundoff decides (VI bar)."""
    idx, kw, min_prefix = TRACE_CASES[tc]
    name, w, var = all_cases[idx]
    fixed = bool(kw.get("fixed_iterations", 0))
    p = vio.BaProblem(w, variant=var, **kw)
    o = oracle_lib.ba_solve(vio, p)
    cloud = oracle_cloud(vio, w, var, **kw)
    solo = gpu_ctx.ba_solve([p])[0]            # cluster route (default for small batches)
    try:
        gpu_ctx.set_ba_route(gpu_ctx.ROUTE_SINGLE_KERNEL)
        mono = gpu_ctx.ba_solve([p])[0]        # single-kernel route
        gpu_ctx.set_ba_route(gpu_ctx.ROUTE_PHASES)
        phases = gpu_ctx.ba_solve([p])[0]      # phase kernels (the route of large batches)
    finally:
        gpu_ctx.set_ba_route(gpu_ctx.ROUTE_AUTO)
    for g in (solo, mono, phases):
        assert len(g["trace"]["cost"]) == g["iterations"]
        compare_traces(o, g, cloud, fixed, min(min_prefix, o["iterations"]))


def test_pnp_trace_rounds(vio, gpu_ctx, all_cases):
    """SolvePnP's four outlier rounds each restart Ceres: the trace holds the rounds one after
    another, iteration numbers restarting at 0, equal to the oracle's (6 parameters: well conditioned)."""
    name, w, var = all_cases[6]
    p = vio.BaProblem(w, variant=var)
    o, g = oracle_lib.ba_solve(vio, p), gpu_ctx.ba_solve([p])[0]
    to, tg = o["trace"], g["trace"]
    assert len(tg["cost"]) == g["iterations"] == o["iterations"] == len(to["cost"])
    assert (to["iteration"] == 0).sum() == 4 and np.array_equal(tg["iteration"], to["iteration"])
    assert np.array_equal(tg["step_is_successful"], to["step_is_successful"])
    assert np.allclose(tg["cost"], to["cost"], rtol=1e-9, atol=0)


def assert_parity_vi_converged(vio, w, o, g, **kw):
    """VI windows with the reference's IMU information (the rotation block of the preintegrated
    covariance is never propagated, IMUPreintegrator.cpp:240-274, so its sqrt-information is 1e4)
    are ill-conditioned near the optimum: the oracle's own answer moves by ~2e-4 m (poses) / ~2e-3 m
    (landmarks) and its iteration count by up to 8 when its landmark inputs move by 1e-15..1e-14
    relative (a few ulp) — the per-iteration traces (test_lm_trace_matches_oracle) show that
    difference growing smoothly from 1e-16 at iteration 0, not a flipped decision.  So for
    tolerance-terminated VI solves the bar is that perturbed-oracle cloud: GPU-vs-oracle
    differences within 2x its largest member's (and within 1e-4 m / 1e-3 m when the cloud is tighter),
    iterations inside the cloud's range +-1, final cost within 2x the cloud's spread or 1e-6."""
    cloud = oracle_cloud(vio, w, vio.VIO_BA_VI, **kw)
    dt_c = max(np.abs(o["T_wb"][:, :3, 3] - c["T_wb"][:, :3, 3]).max() for c in cloud)
    dl_c = max(np.abs(o["lm_xyz"] - c["lm_xyz"]).max() for c in cloud)
    dc_c = max(abs(o["final_cost"] - c["final_cost"]) for c in cloud)
    dr_c = max(rot_angle(o["T_wb"][k, :3, :3], c["T_wb"][k, :3, :3]) for c in cloud for k in range(len(o["T_wb"])))
    dt = np.abs(o["T_wb"][:, :3, 3] - g["T_wb"][:, :3, 3]).max()
    dl = np.abs(o["lm_xyz"] - g["lm_xyz"]).max()
    dc = abs(o["final_cost"] - g["final_cost"])
    assert dt <= max(1e-4, 2 * dt_c), (dt, dt_c)
    assert dl <= max(1e-3, 2 * dl_c), (dl, dl_c)
    assert dc <= max(1e-6 * o["final_cost"], 2 * dc_c), (dc, dc_c)
    for k in range(len(o["T_wb"])):
        assert rot_angle(o["T_wb"][k, :3, :3], g["T_wb"][k, :3, :3]) <= max(1e-5, 2 * dr_c), k
    its = [o["iterations"]] + [c["iterations"] for c in cloud]
    assert min(its) - 1 <= g["iterations"] <= max(its) + 1, (g["iterations"], its)
    assert abs(o["initial_cost"] - g["initial_cost"]) <= 1e-9 * o["initial_cost"]
    assert g["success"] == o["success"] == 1


def config3_cloud():
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "config3_cloud.json")) as f:
        return json.load(f)


# SURVEY §8c's bar per quantity (iterations: +-1)
SURVEY_BAR = {"pos_m": 1e-4, "rot_rad": 1e-5, "lm_m": 1e-3, "vel": 1e-4, "bg": 1e-4, "ba": 1e-4, "cost_rel": 1e-6}


def assert_parity_config3(o, g):
    """Converged config 3 at the reference's options (RunVIBA, Optimizer.cpp:493-724; Ceres tolerances
    trust_region_minimizer.cc:740-760), judged on measured ground: the oracle's own perturbation cloud
    (tests/golden/config3_cloud.json: the same solve with the landmark inputs moved by 1..50 ulp) moves
    the converged positions by up to 2.8e-4 m, landmarks 2.4e-3 m, velocities 1.5e-4, biases 5.9e-4, the
    cost by 4.6e-5 relative and the iteration count over 36..51 -- wider than SURVEY §8c's bar on every
    quantity but the rotations (3.7e-8 rad).  A valid regrouping of the floating-point sums (the GPU's
    fixed-order reductions, another Schur group size) moves the answer the same way, so each quantity is
    held to max(SURVEY bar, 2 x the cloud), the iterations to the cloud's range +-1."""
    cl = config3_cloud()
    K = len(o["T_wb"])
    got = {
        "pos_m": np.abs(o["T_wb"][:, :3, 3] - g["T_wb"][:, :3, 3]).max(),
        "rot_rad": max(rot_angle(o["T_wb"][k, :3, :3], g["T_wb"][k, :3, :3]) for k in range(K)),
        "lm_m": np.abs(o["lm_xyz"] - g["lm_xyz"]).max(),
        "vel": np.abs(o["vel"] - g["vel"]).max(),
        "bg": np.abs(o["bg"] - g["bg"]).max(),
        "ba": np.abs(o["ba"] - g["ba"]).max(),
        "cost_rel": abs(o["final_cost"] - g["final_cost"]) / o["final_cost"],
    }
    lo, hi = cl["iterations_range"]
    print(f"config-3 converged parity: iterations gpu {g['iterations']} oracle {o['iterations']} "
          f"(cloud {lo}..{hi})")
    for k, v in got.items():
        bar = max(SURVEY_BAR[k], 2 * cl["max"][k])
        print(f"  {k:9s} gpu-oracle {v:.3e}  cloud {cl['max'][k]:.3e}  survey {SURVEY_BAR[k]:.0e}  bar {bar:.3e}")
        assert v <= bar, (k, v, bar)
    assert g["success"] == o["success"] == 1
    assert o["iterations"] == cl["oracle"]["iterations"]  # the fixture belongs to this oracle build
    assert lo - 1 <= g["iterations"] <= hi + 1, (g["iterations"], lo, hi)
    assert abs(o["initial_cost"] - g["initial_cost"]) <= 1e-9 * o["initial_cost"]


@pytest.mark.parametrize("idx", range(8))
def test_ba_parity_reference_options(vio, gpu_ctx, all_cases, idx):
    """Reference solver options (50 iterations, Ceres tolerances), every Optimizer variant."""
    name, w, var = all_cases[idx]
    p = vio.BaProblem(w, variant=var)
    o = oracle_lib.ba_solve(vio, p)
    g = gpu_ctx.ba_solve([p])[0]
    if name == "cfg3-vi":
        assert_parity_config3(o, g)
        # besides the wide envelope: the GPU's per-iteration trace equals the oracle's up to the first
        # decision inside the perturbed oracles' margin, and its iteration count lies within the spread of
        # the oracle and the perturbed runs that share that prefix
        cloud = oracle_cloud(vio, w, var)
        stop = compare_traces(o, g, cloud, False, min(30, o["iterations"]))
        its = [o["iterations"]] + [c["iterations"] for c in cloud]
        print(f"config-3 trace prefix {stop}, iterations gpu {g['iterations']}, oracle + cloud {its}")
        assert min(its) - 1 <= g["iterations"] <= max(its) + 1, (g["iterations"], its)
    elif var == vio.VIO_BA_VI:
        assert_parity_vi_converged(vio, w, o, g)
    else:
        assert_parity(o, g, p.c.chi2_threshold)
    if var != vio.VIO_PNP:
        assert g["final_cost"] < g["initial_cost"]


@pytest.mark.parametrize("idx,iters", [(0, 10), (2, 10), (3, 10), (2, 30), (5, 20)])
def test_ba_parity_fixed_iterations(vio, gpu_ctx, all_cases, idx, iters):
    """Benchmark mode (exactly `iters` LM iterations, tolerances off) — the timed configuration, and
    long VI trajectories through accepted and rejected steps."""
    name, w, var = all_cases[idx]
    p = vio.BaProblem(w, variant=var, max_iterations=iters, fixed_iterations=1)
    o = oracle_lib.ba_solve(vio, p)
    g = gpu_ctx.ba_solve([p])[0]
    assert o["iterations"] == g["iterations"] == iters + 1  # iterations.size() counts iteration 0
    assert (o["num_successful_steps"], o["num_unsuccessful_steps"]) == \
        (g["num_successful_steps"], g["num_unsuccessful_steps"])
    assert_parity(o, g, p.c.chi2_threshold, iters_tol=0)


def test_ba_vi_long_fixed_trajectory(vio, gpu_ctx, all_cases):
    """40 fixed LM iterations on a VI window run past convergence, where accept / reject decisions
    are made on roundoff-sized cost changes (from iteration 26 on the decision margins are within
    1e-11 of the cost; the oracle's own perturbed runs flip them too): judged at the perturbed-oracle
    cloud bar, with the iteration count exact."""
    name, w, var = all_cases[5]
    assert var == vio.VIO_BA_VI
    kw = dict(max_iterations=40, fixed_iterations=1)
    p = vio.BaProblem(w, variant=var, **kw)
    o = oracle_lib.ba_solve(vio, p)
    g = gpu_ctx.ba_solve([p])[0]
    assert o["iterations"] == g["iterations"] == 41
    assert_parity_vi_converged(vio, w, o, g, **kw)


def test_batched_equals_single_bitwise(vio, synth, gpu_ctx):
    """Windows are independent: a window's result inside a batch is bitwise its solo result, and
    repeated runs are bitwise identical (fixed-order reductions, no atomics)."""
    ws = [synth.config3(synth.SEED + i) for i in range(6)]
    probs = [vio.BaProblem(w, variant=vio.VIO_BA_VI) for w in ws]
    batch = gpu_ctx.ba_solve(probs)
    batch2 = gpu_ctx.ba_solve(probs)
    for i, p in enumerate(probs):
        solo = gpu_ctx.ba_solve([p])[0]
        for key in ("T_wb", "lm_xyz", "obs_chi2", "vel", "bg", "ba"):
            assert np.array_equal(batch[i][key], solo[key]), (i, key)
            assert np.array_equal(batch[i][key], batch2[i][key]), (i, key)
        assert batch[i]["final_cost"] == solo["final_cost"]


def test_one_shot_arena_reuse_bitwise(vio, synth):
    """vio_ba_solve reuses the context's grow-only device arena and pinned staging buffers from call to call
    (one upload, one download per call): solves of different shapes in a row -- growing, shrinking, and the
    first problem again -- each equal the same window solved as a resident batch (its own allocation), bit
    for bit, and the observation-order outputs land in the caller's order."""
    ctx = vio.Context(0)
    try:
        probs = [vio.BaProblem(synth.config2(), variant=vio.VIO_BA_LOCAL, max_iterations=8, fixed_iterations=1),
                 vio.BaProblem(synth.config3(), variant=vio.VIO_BA_VI, max_iterations=8, fixed_iterations=1),
                 vio.BaProblem(synth.make_window(K=6, L=80, seed=5, marg_frac=0.2, outlier_frac=0.05,
                                                 all_visible=False), variant=vio.VIO_BA_FULL)]
        ref = []
        for p in probs:
            b = vio.BaBatch(ctx, [p])
            b.run()
            b.sync()
            ref.append(b.download()[0])
            b.close()
        for i in (0, 1, 2, 0, 1):
            g = ctx.ba_solve([probs[i]])[0]
            for key in ("T_wb", "lm_xyz", "obs_chi2", "obs_outlier", "lm_bad", "vel", "bg", "ba"):
                assert np.array_equal(g[key], ref[i][key]), (i, key)
            assert g["final_cost"] == ref[i]["final_cost"] and g["iterations"] == ref[i]["iterations"]
        call = ctx.ba_solve_call(probs[1:2])  # the bench's form of the call
        call()
        assert np.array_equal(call.results()[0]["T_wb"], ref[1]["T_wb"])
    finally:
        ctx.close()


def test_routes_agree(vio, synth, gpu_ctx):
    """The single-kernel solver (vio_ctx_set_ba_route) has fixed summation orders that differ from the
    phase kernels': a window of a 40-window single-kernel batch agrees with its solo phase-route result
    to roundoff."""
    ws = [synth.config3(synth.SEED + i) for i in range(40)]
    probs = [vio.BaProblem(w, variant=vio.VIO_BA_VI, max_iterations=10, fixed_iterations=1) for w in ws]
    gpu_ctx.set_ba_route(gpu_ctx.ROUTE_SINGLE_KERNEL)
    try:
        big = gpu_ctx.ba_solve(probs)
    finally:
        gpu_ctx.set_ba_route(gpu_ctx.ROUTE_AUTO)
    for i in (0, 17, 39):
        solo = gpu_ctx.ba_solve([probs[i]])[0]
        assert big[i]["iterations"] == solo["iterations"]
        assert np.abs(big[i]["T_wb"] - solo["T_wb"]).max() <= 1e-7
        assert np.abs(big[i]["lm_xyz"] - solo["lm_xyz"]).max() <= 1e-6
        assert abs(big[i]["final_cost"] - solo["final_cost"]) <= 1e-8 * solo["final_cost"]


def test_cluster_route_bitwise_across_member_counts(vio, synth, gpu_ctx):
    """The cluster route's results do not depend on how many workgroups a window gets: a window solved
    alone (one member workgroup per landmark chunk) and inside a 32-window batch (several chunks per
    member) agree bit for bit (chunk partials and Schur groups are per chunk, summed in chunk order by
    the leader), and a second run of the batch reproduces them."""
    ws = [synth.config3(synth.SEED + i) for i in range(32)]
    probs = [vio.BaProblem(w, variant=vio.VIO_BA_VI, max_iterations=10, fixed_iterations=1) for w in ws]
    gpu_ctx.set_ba_route(gpu_ctx.ROUTE_CLUSTER)  # (auto gives a 32-window batch the phase kernels)
    try:
        big = gpu_ctx.ba_solve(probs)
        big2 = gpu_ctx.ba_solve(probs)
        solos = {i: gpu_ctx.ba_solve([probs[i]])[0] for i in (0, 13, 31)}
    finally:
        gpu_ctx.set_ba_route(gpu_ctx.ROUTE_AUTO)
    for i in (0, 13, 31):
        solo = solos[i]
        for key in ("T_wb", "lm_xyz", "obs_chi2", "vel", "bg", "ba"):
            assert np.array_equal(big[i][key], solo[key]), (i, key)
            assert np.array_equal(big[i][key], big2[i][key]), (i, key)
        assert big[i]["final_cost"] == solo["final_cost"] and big[i]["iterations"] == solo["iterations"]


def test_cluster_and_phase_routes_agree(vio, synth, gpu_ctx):
    """The cluster route (one landmark chunk per Schur group) and the phase kernels (5 chunks per group
    for small batches) sum the Schur partials in different groupings: equal to roundoff on fixed
    10-iteration solves, step decisions identical."""
    ws = [synth.config3(synth.SEED + i) for i in range(4)] + [synth.config2()]
    probs = [vio.BaProblem(w, variant=vio.VIO_BA_VI if i < 4 else vio.VIO_BA_LOCAL, max_iterations=10,
                           fixed_iterations=1) for i, w in enumerate(ws)]
    cl = gpu_ctx.ba_solve(probs)
    gpu_ctx.set_ba_route(gpu_ctx.ROUTE_PHASES)
    try:
        ph = gpu_ctx.ba_solve(probs)
    finally:
        gpu_ctx.set_ba_route(gpu_ctx.ROUTE_AUTO)
    for a, b in zip(cl, ph):
        assert a["iterations"] == b["iterations"]
        assert (a["num_successful_steps"], a["num_unsuccessful_steps"]) == (b["num_successful_steps"],
                                                                           b["num_unsuccessful_steps"])
        assert np.abs(a["T_wb"] - b["T_wb"]).max() <= 1e-7
        assert np.abs(a["lm_xyz"] - b["lm_xyz"]).max() <= 1e-6
        assert abs(a["final_cost"] - b["final_cost"]) <= 1e-8 * b["final_cost"]


def test_mixed_variant_batch(vio, gpu_ctx, all_cases):
    """One launch may mix variants and sizes (LocalBA, BA, VIBA, PnP)."""
    probs = [vio.BaProblem(w, variant=v) for _, w, v in all_cases]
    res = gpu_ctx.ba_solve(probs)
    for p, g in zip(probs, res):
        solo = gpu_ctx.ba_solve([p])[0]
        assert np.array_equal(g["T_wb"], solo["T_wb"])
        assert g["iterations"] == solo["iterations"]


def test_edge_cases(vio, synth, gpu_ctx):
    base = synth.make_window(K=4, L=30, seed=21)
    # (1) no observations: nothing to optimise, poses returned unchanged (Optimizer.cpp:309-333)
    w = dict(base)
    w["obs_kf"] = np.zeros(0, np.int32); w["obs_lm"] = np.zeros(0, np.int32); w["obs_uv"] = np.zeros((0, 2), np.float32)
    p = vio.BaProblem(w, variant=vio.VIO_BA_LOCAL)
    g, o = gpu_ctx.ba_solve([p])[0], oracle_lib.ba_solve(vio, p)
    assert np.allclose(g["T_wb"], o["T_wb"], atol=1e-12) and g["iterations"] == o["iterations"] == 0
    # (2) everything constant: only fixed cost
    w = dict(base)
    w["kf_const"] = np.ones(4, np.uint8); w["lm_const"] = np.ones(30, np.uint8)
    p = vio.BaProblem(w, variant=vio.VIO_BA_LOCAL)
    g, o = gpu_ctx.ba_solve([p])[0], oracle_lib.ba_solve(vio, p)
    assert abs(g["initial_cost"] - o["initial_cost"]) <= 1e-9 * o["initial_cost"]
    assert g["fixed_cost"] > 0 and abs(g["fixed_cost"] - o["fixed_cost"]) <= 1e-9 * o["fixed_cost"]
    # (3) single keyframe window, points free
    w = synth.make_window(K=1, L=20, seed=2)
    p = vio.BaProblem(w, variant=vio.VIO_BA_FULL)
    assert_parity(oracle_lib.ba_solve(vio, p), gpu_ctx.ba_solve([p])[0], p.c.chi2_threshold)
    # (4) invalid arguments fail loudly with the documented error code
    bad = synth.make_window(K=3, L=10, seed=4)
    bad["obs_lm"] = bad["obs_lm"].copy(); bad["obs_lm"][0] = 999
    with pytest.raises(vio.VioError):
        gpu_ctx.ba_solve([vio.BaProblem(bad)])
    # (5) VI windows beyond 10 keyframes: the resident-batch API (windowed path only) refuses them;
    # vio_ba_solve routes them to the global path (test_global_vi_parity)
    with pytest.raises(vio.VioError):
        vio.BaBatch(gpu_ctx, [vio.BaProblem(synth.make_window(K=12, L=10, seed=1, imu=True), variant=vio.VIO_BA_VI)])


def test_config4_full_size_properties(vio, synth, gpu_ctx):
    """256 VIO windows (config 4 shape) in one launch against the oracle's converged results for all
    256 and their perturbation clouds (landmark inputs x (1 + e), e = +-1e-15 .. +-1e-14;
    tests/golden/config4_oracle.json, tests/golden/gen_config4_summary.py): initial costs to 1e-9;
    final costs within 2e-4 of the oracle's or of a cloud member's (the VI windows bifurcate under
    roundoff: window 179 stops after 51 or after 27 iterations, at cost 2814.2 or 2861.55, depending
    on a 1e-15 input change); iteration counts inside the cloud's range +-1; at most 2 windows (<1 %;
    a held-out e = -5e-14 oracle run has 1) outside those bands; the pose error against the synthetic
    truth (final / initial) on average within 0.01 of the oracle's.  Sampled windows at the VI bar,
    fixed-iteration trajectories at the tight bar."""
    import json
    import os
    ref = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "config4_oracle.json")))["windows"]
    ws = synth.config4(256)
    probs = [vio.BaProblem(w, variant=vio.VIO_BA_VI) for w in ws]
    res = gpu_ctx.ba_solve(probs)
    ratio_g, ratio_o, off_cost, off_it = [], [], [], []
    for w, g, r in zip(ws, res, ref):
        assert g["success"] == r["success"] == 1 and g["final_cost"] < 1e-2 * g["initial_cost"]
        assert abs(g["initial_cost"] - r["initial_cost"]) <= 1e-9 * r["initial_cost"], r["window"]
        costs = [r["final_cost"]] + r["cloud_final_cost"]
        its = [r["iterations"]] + r["cloud_iterations"]
        if min(abs(g["final_cost"] - c) / c for c in costs) > 2e-4:
            off_cost.append((r["window"], g["final_cost"], costs))
        if not min(its) - 1 <= g["iterations"] <= max(its) + 1:
            off_it.append((r["window"], g["iterations"], its))
        e0 = np.abs(w["T_wb_init"][:, :3, 3] - w["T_wb_true"][:, :3, 3]).mean()
        e1 = np.abs(g["T_wb"][:, :3, 3] - w["T_wb_true"][:, :3, 3]).mean()
        ratio_g.append(e1 / e0)
        ratio_o.append(r["pose_err_final"] / r["pose_err_init"])
    print(f"config 4 at reference options: windows outside the final-cost band {[o[0] for o in off_cost]}, "
          f"outside the iteration band {[o[0] for o in off_it]}")
    assert len(off_cost) <= 2 and len(off_it) <= 2, (off_cost, off_it)
    ratio_g, ratio_o = np.array(ratio_g), np.array(ratio_o)
    assert abs(ratio_g.mean() - ratio_o.mean()) <= 0.01 and ratio_g.mean() < 0.2
    # converged answers of sampled windows at the VI parity bar (oracle perturbation cloud)
    for i in (0, 255):
        assert_parity_vi_converged(vio, ws[i], oracle_lib.ba_solve(vio, probs[i]), res[i])
    # fixed iterations (the timed configuration): every one of the 256 windows at the tight bar, none
    # allowed outside it (oracle solves over a host thread pool; the ctypes call releases the GIL)
    from concurrent.futures import ThreadPoolExecutor
    fixed = [vio.BaProblem(w, variant=vio.VIO_BA_VI, max_iterations=10, fixed_iterations=1) for w in ws]
    fres = gpu_ctx.ba_solve(fixed)
    with ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
        fora = list(ex.map(lambda p: oracle_lib.ba_solve(vio, p), fixed))
    off = []
    for i, (p, g, o) in enumerate(zip(fixed, fres, fora)):
        try:
            assert_parity(o, g, p.c.chi2_threshold, iters_tol=0)
        except AssertionError as e:
            off.append((i, str(e)[:200]))
    assert not off, off


@pytest.mark.parametrize("K,L", [(16, 200), (40, 300)])
def test_global_vi_parity(vio, synth, gpu_ctx, K, L):
    """RunVIBA beyond the windowed path's 10 keyframes (Optimizer.cpp:493-724: any frames.size() >= 2)
    on the global path (velocities and biases after the poses in the dense reduced system): 10 fixed LM
    iterations at the tight bar with the iteration count and step outcomes exact, velocities / biases
    to 1e-6; the converged solve at the reference's options at the VI bar.

    Parity here is pinned to the oracle only: no reference output or fixture covers a VIBA run with
    more than 10 keyframes.  The oracle's assumptions for it: Ceres SPARSE_SCHUR eliminates the
    landmarks first (Optimizer.cpp:641 leaves the ordering to Ceres, whose automatic ordering puts
    the independent point blocks in the first group), and the IMU factors' pose Jacobians are zero
    (Factors.cpp:1415-1475), so the reduced system is block diagonal between poses and the
    velocity / bias rows."""
    w = synth.make_window(K=K, L=L, seed=40 + K, imu=True, all_visible=False)
    p = vio.BaProblem(w, variant=vio.VIO_BA_VI, max_iterations=10, fixed_iterations=1)
    o = oracle_lib.ba_solve(vio, p)
    g = gpu_ctx.ba_solve([p])[0]
    assert o["iterations"] == g["iterations"] == 11
    assert (o["num_successful_steps"], o["num_unsuccessful_steps"]) == \
        (g["num_successful_steps"], g["num_unsuccessful_steps"])
    assert_parity(o, g, p.c.chi2_threshold, iters_tol=0)
    for key in ("vel", "bg", "ba"):
        assert np.abs(o[key] - g[key]).max() <= 1e-6, key
    p2 = vio.BaProblem(w, variant=vio.VIO_BA_VI)
    o2 = oracle_lib.ba_solve(vio, p2)
    g2 = gpu_ctx.ba_solve([p2])[0]
    assert g2["final_cost"] < g2["initial_cost"]
    assert_parity_vi_converged(vio, w, o2, g2)


@pytest.mark.parametrize("variant", ["full", "local"])
def test_global_ba_parity(vio, synth, gpu_ctx, variant):
    """K > 16 takes the multi-kernel global path (dense Schur + MFMA Cholesky): same parity bar."""
    w = synth.make_global(K=120, L=6000, k_per=10, seed=31)
    if variant == "local":
        rng = np.random.default_rng(4)
        marg = (rng.random(len(w["lm_xyz"])) < 0.1).astype(np.uint8)
        w = dict(w, lm_const=marg, lm_marg=marg)
    p = vio.BaProblem(w, variant=vio.VIO_BA_FULL if variant == "full" else vio.VIO_BA_LOCAL)
    o = oracle_lib.ba_solve(vio, p)
    g = gpu_ctx.ba_solve([p])[0]
    assert_parity(o, g, p.c.chi2_threshold)
    g2 = gpu_ctx.ba_solve([p])[0]
    assert np.array_equal(g["T_wb"], g2["T_wb"]) and np.array_equal(g["lm_xyz"], g2["lm_xyz"])


def test_global_ba_fixed_iterations(vio, synth, gpu_ctx):
    w = synth.make_global(K=64, L=3000, k_per=8, seed=8)
    p = vio.BaProblem(w, variant=vio.VIO_BA_FULL, max_iterations=10, fixed_iterations=1)
    o = oracle_lib.ba_solve(vio, p)
    g = gpu_ctx.ba_solve([p])[0]
    assert o["iterations"] == g["iterations"] == 11
    assert_parity(o, g, p.c.chi2_threshold, iters_tol=0)


def test_global_ba_arena_reuse_bitwise(vio, synth):
    """The global path keeps its device arena, pinned staging buffer, look-ahead stream and the captured
    Cholesky + triangular-solve graph in the context between solves (the graph is replayed while the solve's
    device arguments repeat).  Solves of different shapes in a row -- visual, VI, a larger visual problem and
    the first again -- each equal that problem solved alone on a fresh context, bit for bit."""
    probs = [vio.BaProblem(synth.make_global(K=64, L=3000, k_per=8, seed=8), variant=vio.VIO_BA_FULL,
                           max_iterations=6, fixed_iterations=1),
             vio.BaProblem(synth.make_window(K=16, L=200, seed=56, imu=True, all_visible=False),
                           variant=vio.VIO_BA_VI, max_iterations=6, fixed_iterations=1),
             vio.BaProblem(synth.make_global(K=120, L=6000, k_per=10, seed=31), variant=vio.VIO_BA_FULL,
                           max_iterations=6, fixed_iterations=1)]
    ref = []
    for p in probs:
        c = vio.Context(0)
        ref.append(c.ba_solve([p])[0])
        c.close()
    ctx = vio.Context(0)
    try:
        for i in (0, 1, 2, 0, 2):
            g = ctx.ba_solve([probs[i]])[0]
            for key in ("T_wb", "lm_xyz", "obs_chi2", "obs_outlier", "lm_bad", "vel", "bg", "ba"):
                assert np.array_equal(g[key], ref[i][key]), (i, key)
            assert g["final_cost"] == ref[i]["final_cost"] and g["iterations"] == ref[i]["iterations"]
    finally:
        ctx.close()


def test_config5_full_size_properties(vio, synth, gpu_ctx):
    """Config 5 (1000 KF x 50k landmarks, dense 5994^2 reduced system) at full size: converges,
    improves on the ground truth, bitwise reproducible."""
    w = synth.make_global()
    p = vio.BaProblem(w, variant=vio.VIO_BA_FULL, max_iterations=15)
    g = gpu_ctx.ba_solve([p])[0]
    assert g["success"] == 1 and g["final_cost"] < 0.5 * g["initial_cost"]
    e0 = np.abs(w["T_wb_init"][:, :3, 3] - w["T_wb_true"][:, :3, 3]).mean()
    e1 = np.abs(g["T_wb"][:, :3, 3] - w["T_wb_true"][:, :3, 3]).mean()
    assert e1 < 0.5 * e0
    g2 = gpu_ctx.ba_solve([p])[0]
    assert np.array_equal(g["T_wb"], g2["T_wb"]) and g["final_cost"] == g2["final_cost"]


def test_packed_records_match_download(vio, synth, gpu_ctx):
    """vio_ba_batch_pack (device pack kernel, the config-4 gather payload) decodes through
    vio_ba_record_unpack to exactly the results vio_ba_batch_download returns, outlier flags in the
    caller's observation order; host and device destinations give the same bytes."""
    import torch
    ws = [synth.config3(synth.SEED + i) for i in range(3)]
    ws.append(synth.make_window(K=8, L=150, seed=3, marg_frac=0.2, outlier_frac=0.05, all_visible=False))
    probs = [vio.BaProblem(w, variant=vio.VIO_BA_VI if i < 3 else vio.VIO_BA_LOCAL, max_iterations=6,
                           fixed_iterations=1) for i, w in enumerate(ws)]
    b = vio.BaBatch(gpu_ctx, probs)
    b.run()
    b.sync()
    ref = b.download()
    host = b.pack()
    rb = b.record_bytes()
    assert host.shape == (4, rb) and rb == max(vio.record_bytes(p.K, p.L, p.N) for p in probs)
    dev = torch.zeros((4, rb), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    b.pack(dev.data_ptr())
    b.sync()
    assert np.array_equal(dev.cpu().numpy(), host)
    for r, rec in zip(ref, host):
        u = vio.unpack_record(rec)
        for k in ("T_wb", "lm_xyz", "obs_outlier", "lm_bad", "bg", "ba"):
            assert np.array_equal(u[k], r[k]), k
        for k in ("iterations", "success", "num_inliers", "num_outliers", "num_bad_lm", "final_cost", "initial_cost"):
            assert u[k] == r[k], k
    assert np.array_equal(vio.unpack_record(host[0])["vel"], ref[0]["vel"])
    b.close()


_GBA_AB = r"""
import importlib, sys, numpy as np
sys.path.insert(0, sys.argv[1])
vio = importlib.import_module("360_visual_inertial_odometry_amd")
synth = importlib.import_module("360_visual_inertial_odometry_amd.synth")
ctx = vio.Context(0)
w = synth.make_global(K=120, L=6000, k_per=10, seed=31)
p = vio.BaProblem(w, variant=vio.VIO_BA_FULL, max_iterations=8, fixed_iterations=1)
g = ctx.ba_solve([p])[0]
np.savez(sys.argv[2], T=g["T_wb"], l=g["lm_xyz"], c=np.array([g["final_cost"]]))
ctx.close()
"""


def test_global_ba_solve_paths_bitwise(vio, tmp_path):
    """Every schedule of the global path gives the default's solution bits: the per-step triangular
    solves (VIO_GBA_PERSISTENT_SOLVE=0, the fallback beyond 256 blocks: every row dot reduced the same
    way), separate update / diagonal / panel launches instead of the chained ones (VIO_GBA_FUSE_M=0),
    direct launches instead of the replayed graph (VIO_GBA_GRAPH=0), every trailing update on the
    side stream (VIO_GBA_FUSE_TRAIL=0) and a threshold that puts the larger early updates on the side
    stream and the later ones inside the next step's launch within one factorisation
    (VIO_GBA_FUSE_TRAIL=20: K = 120 has ~12 block columns, updates of up to 66 tiles): each tile
    receives its column updates in column order in all of them."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    variants = [{}, {"VIO_GBA_PERSISTENT_SOLVE": "0"}, {"VIO_GBA_FUSE_M": "0"}, {"VIO_GBA_GRAPH": "0"},
                {"VIO_GBA_FUSE_TRAIL": "0"}, {"VIO_GBA_FUSE_TRAIL": "20"}]
    for i, v in enumerate(variants):
        f = str(tmp_path / f"gba_{i}.npz")
        subprocess.run([sys.executable, "-c", _GBA_AB, root, f], env=dict(os.environ, **v), check=True, timeout=100)
        outs.append(np.load(f))
    a = outs[0]
    for v, b in zip(variants[1:], outs[1:]):
        assert np.array_equal(a["T"], b["T"]) and np.array_equal(a["l"], b["l"]) and np.array_equal(a["c"], b["c"]), v


_TIMEOUT_CHILD = r"""
import importlib, sys, numpy as np
sys.path.insert(0, sys.argv[1])
vio = importlib.import_module("360_visual_inertial_odometry_amd")
synth = importlib.import_module("360_visual_inertial_odometry_amd.synth")
ctx = vio.Context(0)
if sys.argv[2] == "global":
    p = vio.BaProblem(synth.make_global(K=64, L=3000, k_per=10, seed=31), variant=vio.VIO_BA_FULL,
                      max_iterations=3, fixed_iterations=1)
else:
    p = vio.BaProblem(synth.config3(), variant=vio.VIO_BA_VI, max_iterations=5, fixed_iterations=1)
b = None
if sys.argv[2] == "window-batch":  # a reusable batch: its cluster launch replays a captured graph
    b = vio.BaBatch(ctx, [p])
    print("ROUTE0", b.route()[0])

    def solve():
        b.run()
        b.sync()
        return b.download()[0]
else:
    def solve():
        return ctx.ba_solve([p])[0]
first = None
try:
    first = solve()
    print("FIRST-OK")
except vio.VioError as e:
    print("FIRST-ERR", str(e).replace("\n", " "))
if b is not None:
    print("ROUTE1", b.route()[0])
g = solve()   # afterwards: a normal solve (the same batch replayed / the same context)
print("SECOND", g["iterations"], g["final_cost"] < g["initial_cost"])
if first is not None:  # the fallback's result: bitwise the phase route's, on a context of its own
    c2 = vio.Context(0)
    c2.set_ba_route(c2.ROUTE_PHASES)
    ph = c2.ba_solve([p])[0]
    same = all(np.array_equal(first[k], ph[k]) for k in ("T_wb", "lm_xyz", "obs_chi2", "vel", "bg", "ba"))
    print("PHASES-BITWISE", same and first["final_cost"] == ph["final_cost"])
    c2.close()
if b is not None:
    b.close()
ctx.close()
"""


@pytest.mark.parametrize("path,env", [("global", "VIO_GBA_TEST_TIMEOUT"), ("window", "VIO_BA_TEST_CLUSTER_ERR"),
                                      ("window-batch", "VIO_BA_TEST_CLUSTER_ERR")])
def test_wait_timeouts_report_device_errors(vio, path, env):
    """A timed-out inter-workgroup wait is never a failed step or garbage, and the context stays usable: a
    one-shot test hook starts the first launch with the timeout / error word set.  Global BA (Cholesky /
    triangular-solve hand-offs): VIO_EDEVICE, the second solve is normal.  Window BA on the cluster route
    (the members give up at their next wait): the solve falls back to the phase route and returns its result
    bit for bit -- for a one-shot solve, and for a reusable batch, whose cluster launch is a captured graph
    (the hand-off words are cleared outside it, so the hook applies to the first replay) and which stays on
    the phase route afterwards.  The waits themselves are bounded by wall clock (chol_dev.h wait_expired, 2 s)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _TIMEOUT_CHILD, root, path], env=dict(os.environ, **{env: "1"}),
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.split("\n")
    first = [x for x in lines if x.startswith("FIRST")][0]
    second = [x for x in lines if x.startswith("SECOND")][0].split()
    assert second[2] == "True", r.stdout
    if path == "global":
        assert first.startswith("FIRST-ERR") and "(-5)" in first, r.stdout  # VIO_EDEVICE
        return
    assert first == "FIRST-OK", r.stdout
    assert "PHASES-BITWISE True" in lines, r.stdout
    if path == "window-batch":
        assert "ROUTE0 cluster" in lines and "ROUTE1 phases" in lines, r.stdout


def test_batches_from_two_threads(vio, synth):
    """INTEGRATION.md's threading model (one vio_ctx per host thread): two threads, each with its own
    context on device 0, create and run phase-route batches at the same time — the per-device kernel
    attribute set-up (dynamic LDS limits, set once under a lock) must be in place before either
    thread's first launch.  Each thread's results equal the single-threaded solve's, bit for bit."""
    import threading
    probs = [vio.BaProblem(synth.config3(synth.SEED + i), variant=vio.VIO_BA_VI, max_iterations=5,
                           fixed_iterations=1) for i in range(4)]
    ref_ctx = vio.Context(0)
    ref = ref_ctx.ba_solve(probs)
    ref_ctx.close()
    out, err = {}, []

    def work(tid):
        try:
            ctx = vio.Context(0)
            b = vio.BaBatch(ctx, probs[2 * tid:2 * tid + 2])
            for _ in range(3):
                b.run()
            b.sync()
            out[tid] = b.download()
            b.close()
            ctx.close()
        except Exception as e:  # noqa: BLE001 - reported below
            err.append(repr(e))

    ths = [threading.Thread(target=work, args=(t,)) for t in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(120)
    assert not err, err
    for tid in range(2):
        for j, g in enumerate(out[tid]):
            r = ref[2 * tid + j]
            assert np.array_equal(g["T_wb"], r["T_wb"]) and np.array_equal(g["lm_xyz"], r["lm_xyz"]), (tid, j)


def test_cluster_batches_from_two_threads(vio, synth):
    """Two threads, each with its own context on device 0, run 16-window cluster-route batches at the
    same time: each batch alone takes nearly every CU (15 workgroups per window), so without the
    co-residency ledger (residency.h) both launches could be partly placed and wait for each other until
    their bounded waits expire.  The ledger holds the second launch until the first has finished: both
    succeed, bit for bit the single-threaded results."""
    import threading
    probs = [vio.BaProblem(synth.config3(synth.SEED + i), variant=vio.VIO_BA_VI, max_iterations=5,
                           fixed_iterations=1) for i in range(32)]
    ref_ctx = vio.Context(0)
    ref_ctx.set_ba_route(ref_ctx.ROUTE_CLUSTER)
    ref = ref_ctx.ba_solve(probs[:16]) + ref_ctx.ba_solve(probs[16:])
    ref_ctx.close()
    out, err, routes = {}, [], {}
    start = threading.Barrier(2)

    def work(tid):
        try:
            ctx = vio.Context(0)
            ctx.set_ba_route(ctx.ROUTE_CLUSTER)
            b = vio.BaBatch(ctx, probs[16 * tid:16 * tid + 16])
            routes[tid] = b.route()
            start.wait(30)
            for _ in range(3):
                b.run()
            b.sync()
            out[tid] = b.download()
            out[tid, "solve"] = ctx.ba_solve(probs[16 * tid:16 * tid + 16])  # one-shot launches as well
            b.close()
            ctx.close()
        except Exception as e:  # noqa: BLE001 - reported below
            err.append(repr(e))

    ths = [threading.Thread(target=work, args=(t,)) for t in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(120)
    assert not err, err
    for tid in range(2):
        assert routes[tid][0] == "cluster" and routes[tid][1] * 16 > 200, routes[tid]
        for res in (out[tid], out[tid, "solve"]):
            for j, g in enumerate(res):
                r = ref[16 * tid + j]
                assert np.array_equal(g["T_wb"], r["T_wb"]) and np.array_equal(g["lm_xyz"], r["lm_xyz"]), (tid, j)
