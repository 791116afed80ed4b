"""GPU parity of vio_mono_init_solve (csrc/mono_init.hip) against oracle/init_oracle.c.

Initializer::TryMonocularInitialization (src/processing/Initializer.cpp:47-291).  Both sides run the
same f64 Jacobi null vectors / 3x3 SVDs on f32-built systems and the reference's f32 per-point
expressions; the refit sum uses the same fixed order.  Bar (stated here): every integer output
(status, best hypothesis, inlier count and mask, candidate good-point counts, chosen candidate,
triangulated / valid counts) identical; E, R, t, points, scale and the mean reprojection error to
1e-5 relative (device atan2f / asinf vs glibc differ by ulps; the f64 parts are IEEE-exact on both
and agree bitwise in practice).
"""
import numpy as np
import pytest

import init_cases
import oracle_lib

pytestmark = pytest.mark.gpu


def compare(vio, ctx, b1, b2, seed=7, iters=200, **kw):
    P = vio.abi.mono_init_params(ransac_iterations=iters, **kw)
    S = vio.mono_init_samples(seed, len(b1), iters) if iters else np.zeros((0, 8), np.int32)
    g, gm, gX = ctx.mono_init(b1, b2, S, P)
    o, om, oX = oracle_lib.mono_init(vio, b1, b2, S, P)
    for k in ("status", "best_hypothesis", "num_inliers", "pose_candidate", "candidate_good",
              "num_triangulated", "num_valid"):
        assert g[k] == o[k], (k, g[k], o[k])
    np.testing.assert_array_equal(gm, om)
    for k in ("E", "R", "t"):
        d = np.abs(g[k].astype(np.float64) - o[k]).max()
        assert d <= 1e-5 * max(1.0, np.abs(o[k]).max()), (k, d)
    assert abs(g["scale_factor"] - o["scale_factor"]) <= 1e-5 * abs(o["scale_factor"])
    assert abs(g["mean_reproj_error"] - o["mean_reproj_error"]) <= 1e-5 * max(1.0, o["mean_reproj_error"])
    nrm = np.maximum(np.linalg.norm(oX, axis=1), 1e-6)
    assert (np.linalg.norm(gX.astype(np.float64) - oX, axis=1) / nrm).max() <= 1e-5
    return g, o, gX, oX


@pytest.mark.parametrize("seed,noise,outl,n", [(1, 0.0, 0.0, 400), (2, 0.05, 0.0, 1000), (3, 0.02, 0.1, 800),
                                               (4, 0.1, 0.3, 2000), (5, 0.0, 0.0, 4096)])
def test_parity_with_oracle(vio, gpu_ctx, seed, noise, outl, n):
    b1, b2, R, t, _ = init_cases.make_case(n=n, seed=seed, noise_deg=noise, outlier_frac=outl)
    g, o, gX, oX = compare(vio, gpu_ctx, b1, b2, seed=seed)
    if outl == 0.0:
        assert g["status"] == vio.abi.VIO_INIT_OK
    assert gpu_ctx.mono_init_kernel_ms() > 0


def test_reference_config_threshold_and_tight_threshold(vio, gpu_ctx):
    b1, b2, *_ = init_cases.make_case(n=600, seed=11, noise_deg=0.02, outlier_frac=0.2)
    compare(vio, gpu_ctx, b1, b2, seed=3)
    g, *_ = compare(vio, gpu_ctx, b1, b2, seed=3, ransac_threshold=0.01)
    assert g["status"] == vio.abi.VIO_INIT_OK


def test_failure_paths(vio, gpu_ctx):
    A = vio.abi
    b1, b2, *_ = init_cases.make_case(n=300, seed=4)
    assert compare(vio, gpu_ctx, b1[:4], b2[:4], iters=0)[0]["status"] == A.VIO_INIT_TOO_FEW_BEARINGS
    assert compare(vio, gpu_ctx, b1, b2, min_features=301)[0]["status"] == A.VIO_INIT_ESSENTIAL_FAILED
    assert compare(vio, gpu_ctx, b1, b2, iters=0)[0]["status"] == A.VIO_INIT_ESSENTIAL_FAILED
    # validation failure on noisy bearings (a 1e-9 px bar would compare exact-zero errors, where an ulp
    # of atan2f / asinf decides)
    n1, n2, *_ = init_cases.make_case(n=300, seed=12, noise_deg=0.3)
    assert compare(vio, gpu_ctx, n1, n2, max_reprojection_error=0.05)[0]["status"] == A.VIO_INIT_VALIDATION
    c1, c2, *_ = init_cases.make_case(n=300, seed=5, baseline=0.0)
    compare(vio, gpu_ctx, c1, c2)
    # few hypotheses / tiny n
    compare(vio, gpu_ctx, b1[:8], b2[:8], iters=3, min_features=4)


def test_bad_arguments(vio, gpu_ctx):
    b1, b2, *_ = init_cases.make_case(n=50, seed=6)
    S = vio.mono_init_samples(1, 50, 10)
    S[3, 2] = 50  # out of range: rejected on the host before any launch
    with pytest.raises(vio.VioError):
        gpu_ctx.mono_init(b1, b2, S)
    big = np.zeros((4097, 3), np.float32)
    with pytest.raises(vio.VioError):
        gpu_ctx.mono_init(big, big, np.zeros((1, 8), np.int32))


def test_repeatable(vio, gpu_ctx):
    b1, b2, *_ = init_cases.make_case(n=1000, seed=8, noise_deg=0.05, outlier_frac=0.1)
    S = vio.mono_init_samples(9, 1000, 200)
    a = gpu_ctx.mono_init(b1, b2, S)
    b = gpu_ctx.mono_init(b1, b2, S)
    for k in a[0]:
        assert np.array_equal(np.asarray(a[0][k]), np.asarray(b[0][k])), k
    assert np.array_equal(a[2], b[2])
