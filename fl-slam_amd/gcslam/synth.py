"""Synthetic scan / IMU / hypothesis generator for the benchmark configs.

VLP-16-like scans (16 rings x n_az azimuth steps, azimuth-major firing order) ray-cast into a
20 x 20 x 4 m box room with a ground plane, N(0, 1 cm) range noise, per-point time over the
0.1 s sweep and the reference range-sigmoid weights (backend_node.py:448-459). IMU at 200 Hz
padded to 512 slots (backend_node.py:1927-1951). Hypothesis anchors perturbed by N(0, 5 cm) /
N(0, 0.02 rad). Seeds: default_rng(20261015 + scan_idx).

This is input generation only (host NumPy); no hot-path arithmetic lives here.
"""

from __future__ import annotations

import numpy as np

from .constants import (GC_RANGE_WEIGHT_SIGMA, GC_RANGE_WEIGHT_MIN_R, GC_RANGE_WEIGHT_MAX_R,
                        GC_WEIGHT_FLOOR, GC_MAX_IMU_PREINT_LEN, D_Z, T_BASE_LIDAR)

SEED0 = 20261015
SCAN_PERIOD = 0.1
T0_ABS = 1000.0


def range_weights(dist):
    """backend_node.py:448-459 continuous range weighting."""
    a = (dist - GC_RANGE_WEIGHT_MIN_R) / GC_RANGE_WEIGHT_SIGMA
    b = (GC_RANGE_WEIGHT_MAX_R - dist) / GC_RANGE_WEIGHT_SIGMA
    w_raw = (1.0 / (1.0 + np.exp(-a))) * (1.0 / (1.0 + np.exp(-b)))
    return w_raw * (1.0 - GC_WEIGHT_FLOOR) + GC_WEIGHT_FLOOR


def make_scan(scan_idx: int = 0, n_rings: int = 16, n_az: int = 4096, room=(10.0, 10.0, 4.0),
              omega_z: float = 0.3, vel_x: float = 1.0):
    """One synthetic scan plus its IMU window. Returns a dict of float64 / uint8 arrays."""
    rng = np.random.default_rng(SEED0 + scan_idx)
    o = np.asarray(T_BASE_LIDAR[:3], dtype=np.float64)
    el = np.deg2rad(np.linspace(-15.0, 15.0, n_rings))
    az = 2.0 * np.pi * np.arange(n_az) / n_az
    AZ, EL = np.meshgrid(az, el, indexing="ij")  # (n_az, n_rings): azimuth-major
    d = np.stack([np.cos(EL) * np.cos(AZ), np.cos(EL) * np.sin(AZ), np.sin(EL)], -1).reshape(-1, 3)
    hx, hy, hz = room
    with np.errstate(divide="ignore", invalid="ignore"):
        tx = np.where(d[:, 0] > 0, (hx - o[0]) / d[:, 0], (-hx - o[0]) / d[:, 0])
        ty = np.where(d[:, 1] > 0, (hy - o[1]) / d[:, 1], (-hy - o[1]) / d[:, 1])
        tz = np.where(d[:, 2] > 0, (hz - o[2]) / d[:, 2], (0.0 - o[2]) / d[:, 2])
    tt = np.stack([tx, ty, tz], 1)
    tt[~np.isfinite(tt) | (tt <= 0)] = np.inf
    r = tt.min(axis=1) + rng.normal(0.0, 0.01, size=tt.shape[0])
    pts = o[None, :] + r[:, None] * d
    t_start = T0_ABS + SCAN_PERIOD * scan_idx
    az_idx = np.repeat(np.arange(n_az), n_rings)
    ts = t_start + (az_idx / n_az) * SCAN_PERIOD
    w = range_weights(np.linalg.norm(pts - o[None, :], axis=1))
    ring = np.tile(np.arange(n_rings, dtype=np.uint8), n_az)
    tag = np.zeros(pts.shape[0], np.uint8)
    # IMU over [t_last, t_scan] at 200 Hz, padded with zeros (invalid stamps) to 512.
    t_last, t_scan = t_start, t_start + SCAN_PERIOD
    st = np.arange(t_last, t_scan + 1e-9, 1.0 / 200.0)
    M = GC_MAX_IMU_PREINT_LEN
    stamps = np.zeros(M); gyro = np.zeros((M, 3)); accel = np.zeros((M, 3))
    n = st.shape[0]
    stamps[:n] = st
    gyro[:n] = np.array([0.0, 0.0, omega_z]) + rng.normal(0.0, 1e-3, size=(n, 3))
    accel[:n] = np.array([0.0, 0.0, 9.81]) + rng.normal(0.0, 1e-2, size=(n, 3))
    # wheel odometry (backend_node.py:1748-1765): planar constant-twist pose at t_scan relative to
    # the first odom sample, pose cov 1e-2 (trans) / 1e-3 (rot), twist cov 1e-2·I
    t_rel = t_scan - T0_ABS
    yaw = omega_z * t_rel
    odom_pose = np.array([vel_x * np.sin(yaw) / omega_z, vel_x * (1.0 - np.cos(yaw)) / omega_z, 0.0, 0.0, 0.0, yaw])
    odom_pose[0:2] += rng.normal(0.0, 0.01, size=2)
    odom_cov = np.diag([1e-2, 1e-2, 1e-2, 1e-3, 1e-3, 1e-3])
    odom_twist = np.array([vel_x, 0.0, 0.0, 0.0, 0.0, omega_z]) + rng.normal(0.0, 1e-3, size=6)
    odom_twist_cov = 1e-2 * np.eye(6)
    return dict(points=np.ascontiguousarray(pts), timestamps=ts, weights=w, ring=ring, tag=tag,
                imu_stamps=stamps, imu_gyro=gyro, imu_accel=accel, scan_start=t_start,
                scan_end=t_start + SCAN_PERIOD, t_last=t_last, t_scan=t_scan, dt_sec=SCAN_PERIOD,
                odom_pose=odom_pose, odom_cov=odom_cov, odom_twist=odom_twist, odom_twist_cov=odom_twist_cov)


def make_hypotheses(H: int, seed: int = SEED0, prior_precision: float = 1e-6, yaws=None, tilt: float = 0.0):
    """Identity-prior beliefs (belief.py:328-371) with perturbed anchors.

    yaws: optional world yaws (rad) cycled over the hypotheses; each anchor's rotation is then
    Rz(yaw) · Exp(N(0, tilt²) roll/pitch + N(0, 0.02²)) (a robot that has turned around: rotation
    vectors near ±π). Translations stay N(0, 5 cm)."""
    rng = np.random.default_rng(seed + 777)
    X = np.zeros((H, 6))
    X[:, 0:3] = rng.normal(0.0, 0.05, size=(H, 3))
    X[:, 3:6] = rng.normal(0.0, 0.02, size=(H, 3))
    if yaws is not None:
        from scipy.spatial.transform import Rotation
        yaws = np.asarray(yaws, dtype=np.float64)
        pert = X[:, 3:6].copy()
        pert[:, 0:2] += rng.normal(0.0, tilt, size=(H, 2))
        yaw = yaws[np.arange(H) % yaws.shape[0]]
        R = Rotation.from_rotvec(np.stack([np.zeros(H), np.zeros(H), yaw], 1)) * Rotation.from_rotvec(pert)
        X[:, 3:6] = R.as_rotvec()
    L = np.broadcast_to(prior_precision * np.eye(D_Z), (H, D_Z, D_Z)).copy()
    return dict(X_anchor=X, z_lin=np.zeros((H, D_Z)), L=L, h=np.zeros((H, D_Z)),
                stamp=np.zeros(H), weights=np.full(H, 1.0 / H))


def make_io_evidence(H: int, seed: int = SEED0):
    """Synthetic per-hypothesis IMU/odom-branch evidence (L_io, h_io) and its cert scalars.

    Layout of the cert row (10 f64): ess_odom, ess_imu, ess_gyro, sf_odom, sf_imu, sf_gyro,
    exc_dt, exc_ex, nll_sum, trig_sum (see oracle IOEvidence / include/gcslam.h)."""
    rng = np.random.default_rng(seed + 4242)
    diag = np.array([50.0, 50.0, 1e4, 1e3, 1e3, 1e2, 1e2, 1e2, 1e4, 1e4, 1e4, 1e4,
                     1e3, 1e3, 1e3, 1e2, 1e2, 1e2, 1e2, 1e2, 1e2, 1e2])
    L = np.empty((H, D_Z, D_Z)); h = np.empty((H, D_Z)); cert = np.empty((H, 10))
    for k in range(H):
        A = rng.normal(0.0, 1.0, size=(D_Z, D_Z))
        Lk = A @ A.T + np.diag(diag)
        L[k] = 0.5 * (Lk + Lk.T)
        h[k] = L[k] @ rng.normal(0.0, 1e-3, size=D_Z)
        cert[k] = [1.0, 20.0, 1.0, 1.0, 1.0, 1.0, 0.0, 0.0, 0.01, 0.5]
    return L, h, cert


def make_pointcloud2(scan: dict, T_base_lidar=None, time_mode: str = "relative", layout: str = "vlp16",
                     n_nonfinite: int = 0, seed: int = SEED0):
    """The scan as a PointCloud2 message in the Velodyne VLP-16 driver layout (x, y, z, intensity
    f32; ring u16; time f32 relative to the header stamp; point_step 22 — unaligned fields) or
    layout="f64" (x, y, z f64, ring u8, t f64 absolute; point_step 33). Points are expressed in the
    LiDAR frame (inverse of T_base_lidar), so parse + base transform returns the scan.
    time_mode: "relative" (s from the header stamp), "ns" (absolute ns, exercises the 1e-9 rule),
    "none" (no time field). n_nonfinite points get NaN / ±inf coordinates."""
    from .ops.pointcloud import FLOAT32, FLOAT64, UINT8, UINT16, PointCloud2Msg, PointField, _Header, _Stamp
    from scipy.spatial.transform import Rotation
    T = np.asarray(T_BASE_LIDAR if T_base_lidar is None else T_base_lidar, np.float64)
    R = Rotation.from_rotvec(T[3:6]).as_matrix()
    p_lidar = (scan["points"] - T[None, :3]) @ R  # R^T (p - t)
    n = p_lidar.shape[0]
    stamp = float(scan["scan_start"])
    sec = int(np.floor(stamp)); nsec = int(round((stamp - sec) * 1e9))
    hdr = _Header(stamp=_Stamp(sec=sec, nanosec=nsec))
    rng = np.random.default_rng(seed + 99)
    if layout == "vlp16":
        names = ["x", "y", "z", "intensity", "ring"] + ([] if time_mode == "none" else ["time"])
        fmts = ["<f4", "<f4", "<f4", "<f4", "<u2"] + ([] if time_mode == "none" else ["<f4" if time_mode == "relative" else "<f8"])
        offs = [0, 4, 8, 12, 16] + ([] if time_mode == "none" else [18])
        step = 22 if time_mode == "relative" else (26 if time_mode == "ns" else 18)
        types = [FLOAT32, FLOAT32, FLOAT32, FLOAT32, UINT16] + ([] if time_mode == "none" else
                                                             [FLOAT32 if time_mode == "relative" else FLOAT64])
    else:
        names = ["x", "y", "z", "ring"] + ([] if time_mode == "none" else ["t"])
        fmts = ["<f8", "<f8", "<f8", "u1"] + ([] if time_mode == "none" else ["<f8"])
        offs = [0, 8, 16, 24] + ([] if time_mode == "none" else [25])
        step = 33 if time_mode != "none" else 25
        types = [FLOAT64, FLOAT64, FLOAT64, UINT8] + ([] if time_mode == "none" else [FLOAT64])
    arr = np.zeros(n, dtype=np.dtype({"names": names, "formats": fmts, "offsets": offs, "itemsize": step}))
    arr["x"], arr["y"], arr["z"] = p_lidar[:, 0], p_lidar[:, 1], p_lidar[:, 2]
    if "intensity" in names:
        arr["intensity"] = rng.uniform(0, 100, n)
    arr["ring"] = scan["ring"].astype(np.uint16) + (256 if layout == "vlp16" else 0)  # wraps to u8
    if time_mode == "relative":
        arr[names[-1]] = scan["timestamps"] - stamp
    elif time_mode == "ns":
        arr[names[-1]] = scan["timestamps"] * 1e9
    if n_nonfinite:
        idx = rng.choice(n, n_nonfinite, replace=False)
        for k, i in enumerate(idx):
            arr[["x", "y", "z"][k % 3]][i] = [np.nan, np.inf, -np.inf][k % 3]
    fields = [PointField(nm, o, ty) for nm, o, ty in zip(names, offs, types)]
    return PointCloud2Msg(width=n, height=1, point_step=step, fields=fields, data=arr.tobytes(), header=hdr)
