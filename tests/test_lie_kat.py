"""Lie maths pinned by the reference's own known answers: the angle-axis <-> rotation
matrix tests of the vendored Ceres (thirdparty/ceres-solver/internal/ceres/rotation_test.cc:406-617),
restated for the maps the reference computes with them — SO3d::Exp / SO3d::Log
(src/util/LieUtils.cpp:203-273, incl. the theta ~ pi branch :235-268), SE3d::exp (:305-333) and the IMU
factor's log_SO3 (src/optimization/Factors.cpp:1507-1519).

Ceres stores its matrices column-major; the expected matrices below are the row-major transposes.
Tolerances are Ceres' own (kTolerance = 10 eps for matrices, kLooseTolerance = 1e-9 for angle-axis
round trips, eps for the near-zero round trip) wherever the reference's algorithm meets them.  Near pi
it does not: SO3d::Log takes theta = acos((tr R - 1) / 2) (absolute error ~eps / (pi - theta)) and
divides the skew part by 2 sin(theta) of that theta, whose RELATIVE error is then ~eps / (pi - theta)^2.
So AngleAxisToRotationMatrixAndBack is held per trial to max(1e-9, 1e-15 / (pi - |theta|)^2) (one of the
10000 draws, at pi - 1.4e-4, has 2.4e-8: the plain Rodrigues matrix gives 5.9e-8 through the same Log),
and NearPiAngleAxisRoundTrip (theta in [pi - 1e-8, pi)) is a KAT the reference FAILS: where
(tr R - 1) / 2 rounds to -1 the theta ~ pi branch answers (good to 1e-7 here), but where it rounds to
-1 + 1.1e-16, acos gives pi - 1.49e-8 and the generic branch divides the tiny true skew part (2 sin of
the true theta, ~1e-13) by 2 sin(pi - 1.49e-8): the axis comes back scaled down by up to 1e5 (3373 of
the 10000 draws with this platform's libm).  SO3d::Log is reached only by the IMU initialisation's
rotation residuals (Factors.cpp:1235-1241), far from pi, so the restatement keeps the reference's
behaviour; the tests hold the pi-branch draws to 1e-7 and the GPU to the oracle on every draw.

The random trials reproduce the Ceres tests' draws: srand(5) and rand() / RAND_MAX from this
platform's C library, as the tests call them (3 axis draws, then the angle draw, per trial).
"""
import ctypes as C
import math

import numpy as np
import pytest

import oracle_lib

EPS = np.finfo(np.float64).eps
K_TOL = 10 * EPS        # rotation_test.cc:65
K_LOOSE = 1e-9          # rotation_test.cc:68
K_PI = 3.14159265358979323846
N_TRIALS = 10000        # rotation_test.cc:343
NEAR_PI_BAR = 1e-7      # SO3d::Log's own accuracy in [pi - 1e-8, pi) (module docstring)
PROJ_TOL = 12 * EPS     # orthonormality of SVD-projected rotations (is_orthonormal)

# Ceres' expected matrices (column-major in the test), row-major here
R_X_HALF_PI = np.array([[1, 0, 0], [0, 0, -1], [0, 1, 0]], float)          # :426-429
R_Y_PI = np.array([[-1, 0, 0], [0, 1, 0], [0, 0, -1]], float)              # :443-444
R_X_PI = np.array([[1, 0, 0], [0, -1, 0], [0, 0, -1]], float)              # :482-488
R_Z_THIRD_PI = np.array([[0.5, -math.sqrt(3) / 2, 0], [math.sqrt(3) / 2, 0.5, 0], [0, 0, 1]])  # :548-553


def _libc():
    L = C.CDLL("libc.so.6")
    L.rand.restype = C.c_int
    L.srand.argtypes = [C.c_uint]
    return L


def rand_double(L):
    return L.rand() / 2147483647.0  # RandDouble(), rotation_test.cc:59-62 (RAND_MAX of glibc)


def random_axes(kind):
    """The trial inputs of NearPiAngleAxisRoundTrip (:451-476), AngleAxisToRotationMatrixAndBack
    (:564-591) and ...AndBackNearZero (:593-617)."""
    L = _libc()
    L.srand(5)
    out = np.zeros((N_TRIALS, 3))
    for t in range(N_TRIALS):
        a = np.array([rand_double(L) * 2 - 1 for _ in range(3)])
        norm = math.sqrt(float(a @ a))
        if kind == "near_pi":
            theta = K_PI - 1e-8 * rand_double(L)
        elif kind == "any":
            theta = K_PI * 2 * rand_double(L) - K_PI
        else:
            theta = 1e-16 * (K_PI * 2 * rand_double(L) - K_PI)
        out[t] = a * (theta / norm) if kind == "near_pi" else a * theta / norm
    return out


def is_orthonormal(R, tol=10 * EPS):
    """IsOrthonormal (rotation_test.cc:181-203): column dot products summed in Ceres' order.  The
    reference re-projects every SO3d through an SVD (U V^T, LieUtils.cpp:275-288), which adds a
    rounding of its own: on the AndBack draws the oracle's projected Exp reaches 10.5 eps on 1 of 10000
    (the plain Rodrigues form 7 eps), so the random trials use PROJ_TOL for projected rotations."""
    R = np.asarray(R, float)
    for c1 in range(3):
        for c2 in range(3):
            v = 0.0
            for i in range(3):
                v += float(R[i, c1]) * float(R[i, c2])
            if abs((1.0 if c1 == c2 else 0.0) - v) > tol:
                return False
    return True


def angle_axis_delta(a, e):
    """IsNearAngleAxis (rotation_test.cc:141-176): relative difference, sign-free near pi."""
    a, e = np.asarray(a, float), np.asarray(e, float)
    en = np.linalg.norm(e)
    if en == 0:
        return np.linalg.norm(a)
    if abs(en - K_PI) < K_LOOSE:
        return min(np.linalg.norm(a - e), np.linalg.norm(a + e)) / en
    return np.linalg.norm(a - e) / en


# ---- the oracle (CPU): restatement pinned by the KATs ---------------------------------------------------
class OracleLie:
    def __init__(self):
        L = oracle_lib.load()
        vp = C.c_void_p
        L.oracle_so3_exp.argtypes = [vp, vp]
        L.oracle_se3_exp.argtypes = [vp, vp, vp]
        L.oracle_so3d_log.argtypes = [vp, vp]
        L.oracle_imu_log_so3.argtypes = [vp, vp]
        self.L = L

    @staticmethod
    def _p(a):
        return a.ctypes.data_as(C.c_void_p)

    def exp(self, w):
        w = np.ascontiguousarray(w, float)
        R = np.zeros(9)
        self.L.oracle_so3_exp(self._p(w), self._p(R))
        return R.reshape(3, 3)

    def se3(self, xi):
        xi = np.ascontiguousarray(xi, float)
        R, t = np.zeros(9), np.zeros(3)
        self.L.oracle_se3_exp(self._p(xi), self._p(R), self._p(t))
        return R.reshape(3, 3), t

    def log(self, R):
        R = np.ascontiguousarray(R, float).reshape(9)
        w = np.zeros(3)
        self.L.oracle_so3d_log(self._p(R), self._p(w))
        return w

    def imu_log(self, R):
        R = np.ascontiguousarray(R, float).reshape(9)
        w = np.zeros(3)
        self.L.oracle_imu_log_so3(self._p(R), self._p(w))
        return w


@pytest.fixture(scope="module")
def olie():
    return OracleLie()


def test_oracle_exp_known_answers(olie):
    """ZeroAngleAxis / NearZeroAngleAxis / X pi/2 / Y pi / Z pi/3 to rotation matrix (:406-452, :542-557)."""
    for aa, want in (((0, 0, 0), np.eye(3)), ((1e-24, 2e-24, 3e-24), np.eye(3)), ((K_PI / 2, 0, 0), R_X_HALF_PI),
                     ((0, K_PI, 0), R_Y_PI), ((0, 0, K_PI / 3), R_Z_THIRD_PI)):
        R = olie.exp(aa)
        assert is_orthonormal(R), aa
        assert np.abs(R - want).max() <= K_TOL, (aa, R)


def test_oracle_log_round_trips(olie):
    """The round trips of the X / Y / Z tests and AtPiAngleAxisRoundTrip (:478-534): SO3d::Log of the
    exact matrices, then SO3d::Exp of the answer."""
    for aa, R in (((K_PI / 2, 0, 0), R_X_HALF_PI), ((0, K_PI, 0), R_Y_PI), ((0, 0, K_PI / 3), R_Z_THIRD_PI),
                  ((K_PI, 0, 0), R_X_PI)):
        w = olie.log(R)
        assert angle_axis_delta(w, aa) <= K_LOOSE, (aa, w)
        assert np.abs(olie.exp(w) - R).max() <= K_TOL, aa


def round_trip_bar(aa, tol):
    """Per-trial bar of the AndBack round trips: Ceres' tol, widened near pi by SO3d::Log's own
    conditioning (module docstring)."""
    return np.maximum(tol, 1e-15 / np.maximum(K_PI - np.linalg.norm(np.atleast_2d(aa), axis=1), 1e-300) ** 2)


def test_oracle_random_round_trips(olie):
    """AngleAxisToRotationMatrixAndBack (:564-591, |delta| <= 1e-9 per component) and ...NearZero
    (:593-617, <= eps per component), the Ceres tests' own draws."""
    for kind, tol in (("any", K_LOOSE), ("near_zero", EPS)):
        aas = random_axes(kind)
        err = np.zeros(len(aas))
        for i, aa in enumerate(aas):
            R = olie.exp(aa)
            assert is_orthonormal(R, PROJ_TOL)
            err[i] = np.abs(olie.log(R) - aa).max()
        bar = round_trip_bar(aas, tol)
        assert (err <= bar).all(), (kind, err.max(), int((err > tol).sum()))
        assert (err <= tol).sum() >= len(aas) - 1  # only the draw at pi - 1.4e-4 needs the wider bar


def pi_branch(R):
    """Does SO3d::Log take its theta ~ pi branch on R (LieUtils.cpp:223-235)?"""
    c = max(-1.0, min(1.0, (float(R[0, 0]) + float(R[1, 1]) + float(R[2, 2]) - 1.0) * 0.5))
    return abs(math.sin(math.acos(c))) < 1e-10


def test_oracle_near_pi_round_trip(olie):
    """NearPiAngleAxisRoundTrip (:451-476): the draws SO3d::Log answers by its theta ~ pi branch meet
    1e-7; the others are the reference's own failure (module docstring), counted, not asserted."""
    good, failing = [], 0
    for aa in random_axes("near_pi"):
        R = olie.exp(aa)
        d = angle_axis_delta(aa, olie.log(R))
        if pi_branch(R):
            good.append(d)
        elif d > NEAR_PI_BAR:
            failing += 1
    print(f"near-pi round trip: {len(good)} pi-branch draws, worst {max(good):.2e}; "
          f"{failing} generic-branch draws outside the bar (reference behaviour)")
    assert len(good) >= N_TRIALS // 2 and max(good) <= NEAR_PI_BAR


def test_oracle_imu_log(olie):
    """The IMU factor's log_SO3 (the trace formula, no pi branch: Factors.cpp:1507-1519) on the same
    round trips away from pi, and below its 1e-6 small-angle switch."""
    for aa, R in (((K_PI / 2, 0, 0), R_X_HALF_PI), ((0, 0, K_PI / 3), R_Z_THIRD_PI)):
        assert angle_axis_delta(olie.imu_log(R), aa) <= K_LOOSE
    worst = 0.0
    for aa in random_axes("any"):
        if np.linalg.norm(aa) < K_PI - 1e-3:
            worst = max(worst, np.abs(olie.imu_log(olie.exp(aa)) - aa).max())
    assert worst <= K_LOOSE, worst
    small = np.array([2e-7, -1e-7, 3e-7])
    assert np.abs(olie.imu_log(olie.exp(small)) - small).max() <= EPS  # rounding of the O(1) entries of R


def test_oracle_se3_exp(olie):
    """SE3d::exp: rotation = SO3d::Exp(phi); translation = V rho with V = I + (1 - cos)/th^2 P +
    (th - sin)/th^3 P^2, and rho itself below 1e-10 (LieUtils.cpp:305-333)."""
    rho = np.array([0.3, -1.2, 2.0])
    for phi in ((0, 0, 0), (K_PI / 2, 0, 0), (0, 0, K_PI / 3), (0.1, -0.2, 0.3)):
        R, t = olie.se3(np.r_[rho, phi])
        assert np.abs(R - olie.exp(phi)).max() == 0.0
        th = np.linalg.norm(phi)
        if th == 0:
            assert np.array_equal(t, rho)
            continue
        P = np.array([[0, -phi[2], phi[1]], [phi[2], 0, -phi[0]], [-phi[1], phi[0], 0]], float)
        V = np.eye(3) + (1 - math.cos(th)) / th ** 2 * P + (th - math.sin(th)) / th ** 3 * P @ P
        assert np.abs(t - V @ rho).max() <= 1e-14


# ---- the device code the solvers inline (vio_lie_eval) --------------------------------------------------
@pytest.mark.gpu
def test_gpu_lie_known_answers(vio, gpu_ctx, olie):
    """The window factors' SO3d::Exp (no re-projection) and SE3d::exp, the IMU
    factor's log_SO3, and the IMU initialisation's SO3d::Exp + projection / SO3d::Log on the KATs."""
    cx = gpu_ctx
    kat = [((0, 0, 0), np.eye(3)), ((1e-24, 2e-24, 3e-24), np.eye(3)), ((K_PI / 2, 0, 0), R_X_HALF_PI),
           ((0, K_PI, 0), R_Y_PI), ((0, 0, K_PI / 3), R_Z_THIRD_PI)]
    aas = np.array([a for a, _ in kat], float)
    for op in (cx.LIE_SO3_EXP, cx.LIE_SO3D_EXP):
        Rs = cx.lie_eval(op, aas).reshape(-1, 3, 3)
        for (aa, want), R in zip(kat, Rs):
            assert is_orthonormal(R), (op, aa)
            assert np.abs(R - want).max() <= K_TOL, (op, aa, R)
    # SO3d::Log on the exact matrices incl. the pi branch (Y pi, X pi)
    mats = [(R_X_HALF_PI, (K_PI / 2, 0, 0)), (R_Y_PI, (0, K_PI, 0)), (R_Z_THIRD_PI, (0, 0, K_PI / 3)),
            (R_X_PI, (K_PI, 0, 0))]
    ws = cx.lie_eval(cx.LIE_SO3D_LOG, np.array([m.reshape(9) for m, _ in mats]))
    for (m, aa), w in zip(mats, ws):
        assert angle_axis_delta(w, aa) <= K_LOOSE, (aa, w)
        assert np.abs(olie.exp(w) - m).max() <= K_TOL
    # the IMU factor's log on the rotations it can represent
    wi = cx.lie_eval(cx.LIE_IMU_LOG, np.array([R_X_HALF_PI.reshape(9), R_Z_THIRD_PI.reshape(9)]))
    assert angle_axis_delta(wi[0], (K_PI / 2, 0, 0)) <= K_LOOSE
    assert angle_axis_delta(wi[1], (0, 0, K_PI / 3)) <= K_LOOSE
    # SE3d::exp against the oracle's
    xis = np.array([np.r_[[0.3, -1.2, 2.0], phi] for phi in ((0, 0, 0), (K_PI / 2, 0, 0), (0, 0, K_PI / 3),
                                                              (0.1, -0.2, 0.3), (1e-11, 0, 0))])
    g = cx.lie_eval(cx.LIE_SE3_EXP, xis)
    for xi, row in zip(xis, g):
        R, t = olie.se3(xi)
        assert np.abs(row[:9].reshape(3, 3) - R).max() <= 4 * EPS
        assert np.abs(row[9:] - t).max() <= 4 * EPS * max(1.0, np.abs(t).max())


@pytest.mark.gpu
def test_gpu_lie_random_round_trips(vio, gpu_ctx, olie):
    """The Ceres tests' random draws through the device maps: exp -> log round trips at Ceres' bars
    (near pi at the reference algorithm's own accuracy), and the device against the oracle."""
    cx = gpu_ctx
    anyaa, zero, npi = random_axes("any"), random_axes("near_zero"), random_axes("near_pi")
    for aas, tol in ((anyaa, K_LOOSE), (zero, EPS)):
        R_fac = cx.lie_eval(cx.LIE_SO3_EXP, aas)             # the window factors' exp
        R_ini = cx.lie_eval(cx.LIE_SO3D_EXP, aas)            # exp + projection (SO3d)
        back = cx.lie_eval(cx.LIE_SO3D_LOG, R_ini)
        assert (np.abs(back - aas).max(axis=1) <= round_trip_bar(aas, tol)).all()
        for R in R_ini.reshape(-1, 3, 3)[:500]:
            assert is_orthonormal(R, PROJ_TOL)
        for R in R_fac.reshape(-1, 3, 3)[:500]:
            assert is_orthonormal(R)
        # without the projection the factors' exp is orthonormal to roundoff and equal to the oracle's
        # projected SO3d::Exp to a few ulp
        ref = np.array([olie.exp(a).reshape(9) for a in aas[:500]])
        assert np.abs(R_fac[:500] - ref).max() <= 8 * EPS
        assert np.abs(R_ini[:500] - ref).max() <= 8 * EPS
        ok = np.linalg.norm(aas, axis=1) < K_PI - 1e-3
        wi = cx.lie_eval(cx.LIE_IMU_LOG, R_fac[ok])
        assert np.abs(wi - aas[ok]).max() <= tol
    # near pi: SO3d::Log of the oracle's own matrices (same input bits, so the same branch decisions)
    Rs = np.array([olie.exp(a).reshape(9) for a in npi])
    back = cx.lie_eval(cx.LIE_SO3D_LOG, Rs)
    ref = np.array([olie.log(R) for R in Rs])
    assert np.abs(back - ref).max() <= 1e-12 * np.abs(ref).max()
    pib = [pi_branch(R.reshape(3, 3)) for R in Rs]
    assert max(angle_axis_delta(a, b) for a, b, p in zip(npi, back, pib) if p) <= NEAR_PI_BAR
