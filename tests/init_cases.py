"""Synthetic two-view cases for the monocular initialiser (Initializer.cpp): landmarks around the
camera, frame 2 = frame 1 rotated and translated (P2 = R P1 + t, the reference's T_c1c2 convention),
unit f32 bearings, optional angular noise and gross outliers."""
import numpy as np


def rodrigues(w):
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def make_case(n=400, seed=0, noise_deg=0.0, outlier_frac=0.0, baseline=0.3, rot_deg=5.0):
    rng = np.random.default_rng(seed)
    # landmarks on a shell around the camera (360 degrees; |lat| <= 60 deg), range 2..10 m
    lon = rng.uniform(-np.pi, np.pi, n)
    lat = rng.uniform(-np.pi / 3, np.pi / 3, n)
    rr = rng.uniform(2.0, 10.0, n)
    P1 = np.stack([np.cos(lat) * np.sin(lon), -np.sin(lat), np.cos(lat) * np.cos(lon)], 1) * rr[:, None]
    R = rodrigues(rng.normal(size=3) * np.deg2rad(rot_deg) / np.sqrt(3))
    t = rng.normal(size=3)
    t = t / np.linalg.norm(t) * baseline
    P2 = P1 @ R.T + t
    b1 = P1 / np.linalg.norm(P1, axis=1, keepdims=True)
    b2 = P2 / np.linalg.norm(P2, axis=1, keepdims=True)
    if noise_deg > 0:
        for b in (b1, b2):
            b += rng.normal(size=b.shape) * np.deg2rad(noise_deg)
            b /= np.linalg.norm(b, axis=1, keepdims=True)
    n_out = int(round(outlier_frac * n))
    if n_out:
        idx = rng.choice(n, n_out, replace=False)
        v = rng.normal(size=(n_out, 3))
        b2[idx] = v / np.linalg.norm(v, axis=1, keepdims=True)
    return b1.astype(np.float32), b2.astype(np.float32), R, t, P1
