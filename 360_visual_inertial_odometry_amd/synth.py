"""Synthetic ERP+IMU windows for the BASELINE configs, all seeds fixed.

Produces flat window dictionaries that map 1:1 onto vio_ba_problem (include/vio360.h):
poses are the f32 values the reference keeps in Frame (src/database/Frame.h), cast to f64 at
the boundary exactly like `frame->GetTwb().cast<double>()` (src/optimization/Optimizer.cpp:777).

IMU preintegration is a float32 restatement of IMUPreintegrator::Preintegrate /
IntegrateMeasurement / UpdateCovariance (src/processing/IMUPreintegrator.cpp:143-274) with the
default noise values the reference actually uses (:64-67; SetNoiseParameters is never called).
"""
import math

import numpy as np

F32 = np.float32

# extrinsics.T_BC of config/default_config.yaml:57-61
T_BC_CONFIG = np.array([
    [-0.0013741, -0.99974421, -0.02257504, 0.01065397],
    [-0.02183404, -0.02253969, 0.9995075, 0.00614827],
    [-0.99976066, 0.00186632, -0.02179749, 0.01690583],
    [0.0, 0.0, 0.0, 1.0]], dtype=np.float32)

ERP_W, ERP_H = 960, 480           # camera.width/height (config/default_config.yaml:5-6)
BOUNDARY_MARGIN = 20              # camera.boundary_margin
POLAR_RATIO = 0.15                # Camera::CreatePolarMask default (src/database/Camera.h:76)
SEED = 20251205


def t_cb_f32():
    """Frame::SetTBC: m_T_CB = T_BC.inverse() in f32 (src/database/Frame.cpp:90-93)."""
    return np.linalg.inv(T_BC_CONFIG.astype(np.float64)).astype(np.float32)


def rotz(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])


def so3_exp(w):
    th = float(np.linalg.norm(w))
    K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]], dtype=np.float64)
    if th < 1e-12:
        return np.eye(3) + K
    K = K / th
    return np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * (K @ K)


def erp_project(Pc, W, H):
    """ERP projection of camera points (X-right, Y-down, Z-forward), Factors.cpp:402-406."""
    x, y, z = Pc[..., 0], Pc[..., 1], Pc[..., 2]
    L = np.sqrt(x * x + y * y + z * z)
    theta = np.arctan2(x, z)
    phi = -np.arcsin(y / L)
    return np.stack([W * (0.5 + theta / (2 * np.pi)), H * (0.5 - phi / np.pi)], -1)


def pixel_ok(uv, W, H, margin=BOUNDARY_MARGIN, polar=POLAR_RATIO):
    """!IsInPolarRegion && !IsNearBoundary (src/database/Camera.cpp:120-139)."""
    u, v = uv[..., 0], uv[..., 1]
    vr = v / H
    polar_ok = (vr >= polar) & (vr <= 1 - polar)
    bnd_ok = (u >= margin) & (u <= W - margin) & (v >= margin) & (v <= H - margin)
    return polar_ok & bnd_ok


def camera_points(T_wb, T_cb, P):
    """Pc = T_cb * T_wb^-1 * Pw for every (kf, point): returns (K, L, 3)."""
    R = T_wb[:, :3, :3]
    t = T_wb[:, :3, 3]
    Pb = np.einsum("kji,klj->kli", R, P[None] - t[:, None, :])
    return np.einsum("ij,klj->kli", T_cb[:3, :3], Pb) + T_cb[:3, 3]


# --------------------------------------------------------------------------------------------
# trajectory of configs 2-4: KF i at t = 0.25 i s; p = (0.15 i, 0.03 sin 0.7 i, 0.02 cos 0.5 i),
# yaw 2 deg per KF.  Continuous form in t (s): tau = t / 0.25.
KF_DT = 0.25


def traj_pos(t):
    tau = t / KF_DT
    return np.array([0.15 * tau, 0.03 * math.sin(0.7 * tau), 0.02 * math.cos(0.5 * tau)])


def traj_acc(t):
    s = 1.0 / KF_DT
    tau = t / KF_DT
    return np.array([0.0, -0.03 * 0.49 * s * s * math.sin(0.7 * tau), -0.02 * 0.25 * s * s * math.cos(0.5 * tau)])


def traj_vel(t):
    s = 1.0 / KF_DT
    tau = t / KF_DT
    return np.array([0.15 * s, 0.03 * 0.7 * s * math.cos(0.7 * tau), -0.02 * 0.5 * s * math.sin(0.5 * tau)])


YAW_RATE = math.radians(2.0) / KF_DT


def traj_rot(t):
    return rotz(YAW_RATE * t)


# --------------------------------------------------------------------------------------------
# IMU preintegration, float32 restatement of src/processing/IMUPreintegrator.cpp:143-274
def _skew32(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]], dtype=F32)


def _rodrigues32(w):
    th = F32(np.sqrt(np.sum(w * w, dtype=F32)))
    if th < F32(1e-6):
        return np.eye(3, dtype=F32) + _skew32(w)
    K = _skew32((w / th).astype(F32))
    return (np.eye(3, dtype=F32) + F32(np.sin(th)) * K + (F32(1) - F32(np.cos(th))) * (K @ K)).astype(F32)


def _right_jac32(w):
    th = F32(np.sqrt(np.sum(w * w, dtype=F32)))
    if th < F32(1e-6):
        return (np.eye(3, dtype=F32) - F32(0.5) * _skew32(w)).astype(F32)
    K = _skew32((w / th).astype(F32))
    return (np.eye(3, dtype=F32) - ((F32(1) - F32(np.cos(th))) / th) * K + ((th - F32(np.sin(th))) / th) * (K @ K)).astype(F32)


def preintegrate(samples, start, end, gyro_bias=None, accel_bias=None,
                 gyro_noise=1e-4, accel_noise=1e-3, gyro_bias_noise=1e-6, accel_bias_noise=1e-5):
    """samples: array (M, 7) of [t, ax, ay, az, gx, gy, gz] (the IMUData fields)."""
    gb = np.zeros(3, F32) if gyro_bias is None else np.asarray(gyro_bias, F32)
    ab = np.zeros(3, F32) if accel_bias is None else np.asarray(accel_bias, F32)
    sel = samples[(samples[:, 0] >= start) & (samples[:, 0] < end)]
    if len(sel) == 0:
        return None
    dR = np.eye(3, dtype=F32)
    dV = np.zeros(3, F32)
    dP = np.zeros(3, F32)
    JRg = np.zeros((3, 3), F32)
    JVg = np.zeros((3, 3), F32)
    JVa = np.zeros((3, 3), F32)
    JPg = np.zeros((3, 3), F32)
    JPa = np.zeros((3, 3), F32)
    cov = np.zeros((15, 15), F32)
    dt_total = 0.0
    for i in range(len(sel)):
        if i == 0:
            dt = F32(sel[1, 0] - sel[0, 0]) if len(sel) > 1 else F32(0.002)
        else:
            dt = F32(sel[i, 0] - sel[i - 1, 0])
        dt = F32(max(F32(0.0005), min(dt, F32(0.02))))
        acc = sel[i, 1:4].astype(F32) - ab
        gyr = sel[i, 4:7].astype(F32) - gb
        R, V, P = dR, dV, dP
        wdt = (gyr * dt).astype(F32)
        dRi = _rodrigues32(wdt)
        Jr = _right_jac32(wdt)
        JRg = (-(dRi.T @ Jr) * dt).astype(F32)
        JVg = (JVg + JVa @ _skew32(acc) @ JRg).astype(F32)
        JPg = (JPg + JPa @ _skew32(acc) @ JRg + JVg * dt).astype(F32)
        dR = (R @ dRi).astype(F32)
        dVi = ((R @ acc) * dt).astype(F32)
        dV = (V + dVi).astype(F32)
        JVa = (JVa + R * dt).astype(F32)
        dPi = (V * dt + F32(0.5) * (R @ acc) * dt * dt).astype(F32)
        dP = (P + dPi).astype(F32)
        JPa = (JPa + JVa * dt + F32(0.5) * R * dt * dt).astype(F32)
        # UpdateCovariance (uses the updated delta_R)
        Nga = np.zeros((6, 6), F32)
        Nga[:3, :3] = np.eye(3, dtype=F32) * F32(gyro_noise * gyro_noise)
        Nga[3:, 3:] = np.eye(3, dtype=F32) * F32(accel_noise * accel_noise)
        walk = np.zeros((6, 6), F32)
        walk[:3, :3] = np.eye(3, dtype=F32) * F32(gyro_bias_noise * gyro_bias_noise) * dt
        walk[3:, 3:] = np.eye(3, dtype=F32) * F32(accel_bias_noise * accel_bias_noise) * dt
        A = np.eye(9, dtype=F32)
        B = np.zeros((9, 6), F32)
        A[6:9, 3:6] = np.eye(3, dtype=F32) * dt
        B[3:6, 3:6] = dR * dt
        B[6:9, 3:6] = F32(0.5) * dR * dt * dt
        cov[:9, :9] = (A @ cov[:9, :9] @ A.T + B @ Nga @ B.T).astype(F32)
        cov[9:, 9:] = (cov[9:, 9:] + walk).astype(F32)
        dt_total += float(dt)
    return {"delta_R": dR, "delta_V": dV, "delta_P": dP, "J_Rg": JRg, "J_Vg": JVg, "J_Va": JVa,
            "J_Pg": JPg, "J_Pa": JPa, "cov": cov, "gyro_bias": gb, "accel_bias": ab, "dt_total": dt_total}


def imu_samples(t0, t1, rate, rng, sigma_g, sigma_a, gravity):
    ts = np.arange(int(round(t0 * rate)), int(round(t1 * rate)) + 1) / rate
    out = np.zeros((len(ts), 7))
    w_body = np.array([0.0, 0.0, YAW_RATE])
    for i, t in enumerate(ts):
        R = traj_rot(t)
        f = R.T @ (traj_acc(t) - gravity)
        out[i, 0] = t
        out[i, 1:4] = f + rng.normal(0, sigma_a, 3)
        out[i, 4:7] = w_body + rng.normal(0, sigma_g, 3)
    return out


# --------------------------------------------------------------------------------------------
def make_window(K=10, L=200, seed=SEED, W=ERP_W, H=ERP_H, noise_px=0.5, rot_sigma_deg=0.3,
                trans_sigma=0.02, lm_sigma=0.05, imu=False, marg_frac=0.0, outlier_frac=0.0,
                all_visible=True):
    """Config 2 (imu=False, L=200) / config 3 (imu=True, L=500) window."""
    rng = np.random.default_rng(seed)
    T_cb = t_cb_f32().astype(np.float64)
    T_true = np.zeros((K, 4, 4))
    for i in range(K):
        t = KF_DT * i
        T_true[i, :3, :3] = traj_rot(t)
        T_true[i, :3, 3] = traj_pos(t)
        T_true[i, 3, 3] = 1.0
    # landmarks: bearing in the middle KF's camera with |lat| <= 50 deg, range U[3, 12]
    mid = K // 2
    T_wc_mid = T_true[mid] @ np.linalg.inv(T_cb)
    pts = []
    while len(pts) < L:
        m = 4 * (L - len(pts)) + 16
        lon = rng.uniform(-np.pi, np.pi, m)
        lat = rng.uniform(-np.radians(50), np.radians(50), m)
        rng_m = rng.uniform(3.0, 12.0, m)
        b = np.stack([np.cos(lat) * np.sin(lon), -np.sin(lat), np.cos(lat) * np.cos(lon)], -1)
        Pc = b * rng_m[:, None]
        Pw = Pc @ T_wc_mid[:3, :3].T + T_wc_mid[:3, 3]
        uv = erp_project(camera_points(T_true, T_cb, Pw), W, H)
        ok = pixel_ok(uv, W, H).all(0) if all_visible else pixel_ok(uv, W, H).sum(0) >= 2
        for j in np.nonzero(ok)[0]:
            if len(pts) < L:
                pts.append(Pw[j])
    P_true = np.array(pts)
    uv_true = erp_project(camera_points(T_true, T_cb, P_true), W, H)  # (K, L, 2)
    vis = pixel_ok(uv_true, W, H)
    obs_kf, obs_lm, obs_uv = [], [], []
    for l in range(L):
        for k in range(K):
            if vis[k, l]:
                obs_kf.append(k)
                obs_lm.append(l)
                obs_uv.append(uv_true[k, l] + rng.normal(0, noise_px, 2))
    obs_uv = np.array(obs_uv, dtype=np.float32)
    N = len(obs_kf)
    if outlier_frac > 0:
        bad = rng.random(N) < outlier_frac
        obs_uv[bad] += rng.normal(0, 15.0, (int(bad.sum()), 2)).astype(np.float32)
    # perturbed initial state (KF 0 exact), stored as f32 like Frame / MapPoint
    T_init = T_true.copy()
    for i in range(1, K):
        dR = so3_exp(rng.normal(0, np.radians(rot_sigma_deg), 3))
        T_init[i, :3, :3] = T_true[i, :3, :3] @ dR
        T_init[i, :3, 3] = T_true[i, :3, 3] + rng.normal(0, trans_sigma, 3)
    T_init = T_init.astype(np.float32).astype(np.float64)
    P_init = (P_true + rng.normal(0, lm_sigma, P_true.shape)).astype(np.float32).astype(np.float64)
    kf_const = np.zeros(K, np.uint8)
    kf_const[0] = 1
    lm_marg = (rng.random(L) < marg_frac).astype(np.uint8)
    w = {
        "cols": W, "rows": H, "T_cb": T_cb, "T_wb_init": T_init, "T_wb_true": T_true,
        "kf_const": kf_const, "lm_const": lm_marg.copy(), "lm_marg": lm_marg,
        "lm_xyz": P_init, "lm_true": P_true,
        "obs_kf": np.array(obs_kf, np.int32), "obs_lm": np.array(obs_lm, np.int32), "obs_uv": obs_uv,
    }
    if imu:
        gravity = np.array([0.0, 0.0, -9.81])
        samples = imu_samples(0.0, KF_DT * (K - 1) + 0.01, 200.0, rng, 1e-3, 1e-2, gravity)
        preint = [None]
        for i in range(1, K):
            preint.append(preintegrate(samples, KF_DT * (i - 1), KF_DT * i))
        v_true = np.array([traj_vel(KF_DT * i) for i in range(K)])
        w.update({
            "preint": preint, "gravity": gravity, "imu_samples": samples,
            "vel": (v_true + rng.normal(0, 0.05, v_true.shape)).astype(np.float32).astype(np.float64),
            "bg": np.zeros(3), "ba": np.zeros(3), "vel_true": v_true,
        })
    return w


def config2(seed=SEED):
    return make_window(K=10, L=200, seed=seed)


def config3(seed=SEED):
    return make_window(K=10, L=500, seed=seed, imu=True)


def config4(n=256, seed=SEED):
    return [config3(seed + w) for w in range(n)]


def make_pnp(window, kf=None, seed=SEED + 7, outlier_frac=0.0, marg_frac=0.0):
    """Pose-only problem of one keyframe against fixed landmarks (SolvePnP, Optimizer.cpp:83-302).
    Landmarks fixed at their true positions; the frame starts from the perturbed pose."""
    rng = np.random.default_rng(seed)
    K = len(window["T_wb_init"])
    kf = K - 1 if kf is None else kf
    sel = window["obs_kf"] == kf
    lms = window["obs_lm"][sel]
    uv = window["obs_uv"][sel].copy()
    if outlier_frac > 0:
        bad = rng.random(len(uv)) < outlier_frac
        uv[bad] += rng.normal(0, 20.0, (int(bad.sum()), 2)).astype(np.float32)
    marg = (rng.random(len(lms)) < marg_frac).astype(np.uint8)
    return {
        "cols": window["cols"], "rows": window["rows"], "T_cb": window["T_cb"][None],
        "T_wb_init": window["T_wb_init"][kf][None], "kf_const": np.zeros(1, np.uint8),
        "lm_const": marg, "lm_marg": marg,
        "lm_xyz": window["lm_true"][lms].astype(np.float32).astype(np.float64),
        "obs_kf": np.zeros(len(lms), np.int32), "obs_lm": np.arange(len(lms), dtype=np.int32),
        "obs_uv": uv,
    }


def make_global(K=1000, L=50000, k_per=10, seed=SEED + 5, W=ERP_W, H=ERP_H):
    """Config 5: K KFs on a 4 m circle (0.36 deg/KF), L points on a 10 m cylinder |z|<=3,
    each seen by k_per KFs drawn without replacement among valid ones."""
    rng = np.random.default_rng(seed)
    T_cb = t_cb_f32().astype(np.float64)
    T_true = np.zeros((K, 4, 4))
    for i in range(K):
        a = np.radians(0.36 * i)
        T_true[i, :3, :3] = rotz(a)
        T_true[i, :3, 3] = [4 * math.cos(a), 4 * math.sin(a), 0.0]
        T_true[i, 3, 3] = 1
    ang = rng.uniform(0, 2 * np.pi, L)
    z = rng.uniform(-3, 3, L)
    P = np.stack([10 * np.cos(ang), 10 * np.sin(ang), z], -1)
    obs_kf, obs_lm, obs_uv = [], [], []
    keep = []
    B = 2000
    for l0 in range(0, L, B):
        Pb = P[l0:l0 + B]
        uv = erp_project(camera_points(T_true, T_cb, Pb), W, H)
        ok = pixel_ok(uv, W, H)
        for j in range(len(Pb)):
            cand = np.nonzero(ok[:, j])[0]
            if len(cand) < k_per:
                continue
            ks = np.sort(rng.choice(cand, k_per, replace=False))
            li = len(keep)
            keep.append(l0 + j)
            for k in ks:
                obs_kf.append(k)
                obs_lm.append(li)
                obs_uv.append(uv[k, j] + rng.normal(0, 0.5, 2))
    P_true = P[keep]
    Lk = len(keep)
    T_init = T_true.copy()
    for i in range(1, K):
        T_init[i, :3, :3] = T_true[i, :3, :3] @ so3_exp(rng.normal(0, np.radians(0.3), 3))
        T_init[i, :3, 3] += rng.normal(0, 0.02, 3)
    kf_const = np.zeros(K, np.uint8)
    kf_const[0] = 1
    return {
        "cols": W, "rows": H, "T_cb": T_cb, "T_wb_init": T_init.astype(np.float32).astype(np.float64),
        "T_wb_true": T_true, "kf_const": kf_const, "lm_const": np.zeros(Lk, np.uint8),
        "lm_marg": np.zeros(Lk, np.uint8),
        "lm_xyz": (P_true + rng.normal(0, 0.05, P_true.shape)).astype(np.float32).astype(np.float64),
        "lm_true": P_true, "obs_kf": np.array(obs_kf, np.int32), "obs_lm": np.array(obs_lm, np.int32),
        "obs_uv": np.array(obs_uv, np.float32),
    }


# --------------------------------------------------------------------------------------------
# Config 1: ERP frames of a procedural environment: seeded multi-octave 3-D value
# noise sampled along every ERP ray.  A pure camera rotation gives an analytic flow field.
def _value_noise_tables(seed):
    rng = np.random.default_rng(seed)
    perm = rng.permutation(256).astype(np.int64)
    vals = rng.random(256).astype(np.float32)
    return np.concatenate([perm, perm]), vals


def erp_rays(W, H):
    """Unit bearings of the pixel centres of a W x H ERP image (Camera::PixelToBearing convention:
    X-right, Y-down, Z-forward; u = W(0.5 + lon/2pi), v = H(0.5 - lat/pi)), shape (H, W, 3)."""
    u = (np.arange(W, dtype=np.float64) + 0.5) / W
    v = (np.arange(H, dtype=np.float64) + 0.5) / H
    lon = (u - 0.5) * 2 * np.pi
    lat = -(v - 0.5) * np.pi
    cl = np.cos(lat)[:, None]
    return np.stack([cl * np.sin(lon)[None, :], np.broadcast_to(-np.sin(lat)[:, None], (H, W)),
                     cl * np.cos(lon)[None, :]], -1)


def render_erp(W, H, R_wc=None, seed=1, octaves=6, base_freq=None, rows_per_chunk=64):
    """u8 ERP image of the value-noise environment seen by a camera with rotation R_wc.  The base
    frequency scales with the width so the per-pixel texture (and the LK minEig test) is the same
    at every resolution."""
    if base_freq is None:
        base_freq = 12.0 * W / 960.0
    perm, vals = _value_noise_tables(seed)
    R = np.eye(3) if R_wc is None else np.asarray(R_wc, np.float64)
    img = np.empty((H, W), np.uint8)
    rays_all = erp_rays(W, H)
    for y0 in range(0, H, rows_per_chunk):
        d = rays_all[y0:y0 + rows_per_chunk] @ R.T  # world directions
        acc = np.zeros(d.shape[:2], np.float64)
        amp, tot = 1.0, 0.0
        for o in range(octaves):
            p = d * (base_freq * (2.0 ** o)) + 17.0 * (o + 1)
            i0 = np.floor(p).astype(np.int64)
            f = p - i0
            f = f * f * (3 - 2 * f)  # smoothstep
            n = 0.0
            for dz in (0, 1):
                for dy in (0, 1):
                    for dx in (0, 1):
                        h = perm[(perm[(perm[(i0[..., 0] + dx) & 255] + i0[..., 1] + dy) & 255] + i0[..., 2] + dz) & 255]
                        wgt = (f[..., 0] if dx else 1 - f[..., 0]) * (f[..., 1] if dy else 1 - f[..., 1]) * \
                              (f[..., 2] if dz else 1 - f[..., 2])
                        n = n + wgt * vals[h]
            acc += amp * n
            tot += amp
            amp *= 0.55
        img[y0:y0 + rows_per_chunk] = np.clip(acc / tot * 255.0 * 1.6 - 80.0, 0, 255).astype(np.uint8)
    return img


def rot_yaw_pitch(yaw_deg, pitch_deg):
    """Camera rotation: yaw about camera Y (down axis), then pitch about camera X."""
    a, b = math.radians(yaw_deg), math.radians(pitch_deg)
    Ry = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
    Rx = np.array([[1, 0, 0], [0, math.cos(b), -math.sin(b)], [0, math.sin(b), math.cos(b)]])
    return Ry @ Rx


def erp_flow_truth(pts, W, H, R_21):
    """Analytic position in frame 2 of frame-1 pixels under a pure rotation: d2 = R_21 d1."""
    pts = np.asarray(pts, np.float64)
    lon = (pts[:, 0] / W - 0.5) * 2 * np.pi
    lat = -(pts[:, 1] / H - 0.5) * np.pi
    d = np.stack([np.cos(lat) * np.sin(lon), -np.sin(lat), np.cos(lat) * np.cos(lon)], -1) @ np.asarray(R_21).T
    u = W * (0.5 + np.arctan2(d[:, 0], d[:, 2]) / (2 * np.pi))
    v = H * (0.5 - (-np.arcsin(np.clip(d[:, 1], -1, 1))) / np.pi)
    return np.stack([u, v], -1)


def config1(W=3840, H=1920, yaw_deg=1.5, pitch_deg=0.5, seed=1):
    """Two-frame ERP KLT pair: frame 2 = same scene, camera yawed/pitched (pure rotation).
    Returns (img1, img2, R_21) with R_21 mapping frame-1 camera bearings to frame-2 bearings."""
    R1 = np.eye(3)
    R2 = rot_yaw_pitch(yaw_deg, pitch_deg)  # R_wc of frame 2
    img1 = render_erp(W, H, R1, seed=seed)
    img2 = render_erp(W, H, R2, seed=seed)
    return img1, img2, R2.T @ R1
