"""Synthetic two-view triangulation cases (shared by the CPU oracle test and the GPU parity test)."""
import numpy as np


def _rot(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def make_case(n=4096, n_poses=16, seed=0, baseline=0.5, noise=0.0):
    """Keyframes on a short track (world-to-camera f32), random points 2-20 m away, exact (or
    noisy) unit bearings; candidate i pairs two random distinct keyframes."""
    rng = np.random.default_rng(seed)
    T = np.zeros((n_poses, 4, 4), np.float32)
    centers = np.cumsum(rng.normal(0, baseline, (n_poses, 3)), 0)
    for k in range(n_poses):
        R = _rot(rng)
        T[k, :3, :3] = R
        T[k, :3, 3] = -R @ centers[k]
        T[k, 3, 3] = 1
    pairs = np.zeros((n, 2), np.int32)
    pairs[:, 0] = rng.integers(0, n_poses, n)
    pairs[:, 1] = (pairs[:, 0] + rng.integers(1, n_poses, n)) % n_poses
    mid = 0.5 * (centers[pairs[:, 0]] + centers[pairs[:, 1]])
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    X = mid + d * rng.uniform(2, 20, (n, 1))
    B = np.zeros((n, 6), np.float32)
    for j in range(2):
        Tj = T[pairs[:, j]].astype(np.float64)
        pc = np.einsum("nij,nj->ni", Tj[:, :3, :3], X) + Tj[:, :3, 3]
        pc += rng.normal(0, noise, pc.shape) * np.linalg.norm(pc, axis=1, keepdims=True)
        B[:, 3 * j:3 * j + 3] = (pc / np.linalg.norm(pc, axis=1, keepdims=True)).astype(np.float32)
    return T, pairs, B, X
