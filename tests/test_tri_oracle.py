"""CPU checks of the triangulation oracle (oracle/tri_oracle.py), SURVEY §8 f2:
Estimator::TriangulateSinglePoint (src/processing/Estimator.cpp:1082-1137).  The reference has no
test for it; the oracle is pinned by exact synthetic geometry."""
import importlib.util
import os

import numpy as np

import tri_cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_oracle():
    spec = importlib.util.spec_from_file_location("tri_oracle", os.path.join(ROOT, "oracle", "tri_oracle.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_exact_bearings_recover_points():
    tri = load_oracle()
    T, pairs, B, X = tri_cases.make_case(n=2000, seed=1)
    P, valid, err = tri.triangulate(T, pairs, B, 3840)
    assert valid.all()
    rel = np.linalg.norm(P - X, axis=1) / np.linalg.norm(X, axis=1)
    assert np.median(rel) < 1e-5 and np.percentile(rel, 99) < 1e-3, (np.median(rel), rel.max())
    assert np.median(err) < 0.05


def test_noisy_bearings_reprojection_error_scale():
    tri = load_oracle()
    T, pairs, B, X = tri_cases.make_case(n=2000, seed=2, noise=1e-3)
    P, valid, err = tri.triangulate(T, pairs, B, 3840)
    # 1 mrad of bearing noise ~ 0.6 px at 3840 px / 2π; the DLT residual stays at that scale
    assert np.median(err) < 2.0


def test_row_construction_matches_reference_expression():
    tri = load_oracle()
    T, pairs, B, _ = tri_cases.make_case(n=4, seed=3)
    A = tri.build_A(T[pairs[:, 0]], T[pairs[:, 1]], B[:, :3], B[:, 3:])
    b = B[0]
    T1 = T[pairs[0, 0]]
    np.testing.assert_array_equal(A[0, 0], np.float32(b[0]) * T1[2] - np.float32(b[2]) * T1[0])
    np.testing.assert_array_equal(A[0, 1], np.float32(b[1]) * T1[2] - np.float32(b[2]) * T1[1])


def test_empty():
    tri = load_oracle()
    P, v, e = tri.triangulate(np.eye(4)[None], np.zeros((0, 2)), np.zeros((0, 6)), 960)
    assert P.shape == (0, 3) and v.shape == (0,)
