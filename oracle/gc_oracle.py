"""
TEST INFRASTRUCTURE ONLY — CPU oracle for the GC-SLAM v2 per-scan hot path.

This module is a NumPy restatement of the reference's algorithm (whabacivch/FL-SLAM,
GC-SLAM v2), written from the reference semantics; every function cites the reference
file:line it follows (paths relative to the reference root; ``fl_slam_poc/`` means
``fl_ws/src/fl_slam_poc/fl_slam_poc/``).

Who may use it: ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg — as the checker / the timed CPU baseline, never as the thing
measured or shipped. The product path (``fl-slam_amd/gcslam``) never imports it and
fails loudly when its HIP library is missing.

Pinning: the reference's Python path imports JAX, which is absent from this image;
no stand-in for JAX is used. The oracle is pinned against the
known-answer and property tests the reference's own test suites hold for this path
(``tests/test_oracle_kat.py``, citing each reference test). Rows the reference never
pinned (τ, the legacy bin-path wiring, PoseCovInflationPushforward) are marked
"parity unpinned" where they are defined.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
from scipy.linalg import solve_triangular
from scipy.special import expit

# ---------------------------------------------------------------------------------------
# Constants — fl_slam_poc/common/constants.py:54-143, :259-281 ; pipeline.py:96-160
# ---------------------------------------------------------------------------------------
D_Z = 22
EPS_PSD = 1e-12
EPS_LIFT = 1e-9
EPS_MASS = 1e-12
EPS_R = 1e-6
EXC_EPS = 1e-12
F64_EPS = float(np.finfo(np.float64).eps)
GRAVITY_W = np.array([0.0, 0.0, -9.81])
KAPPA_R0 = 0.8
KAPPA_TAU = 0.03
ALPHA_MIN = 1.0
ALPHA_MAX = 1.0
C0_COND = 1e6
C_FROB = 1.0
ANCHOR_M0 = 0.5
ANCHOR_R0 = 0.2
TIME_WARP_SIGMA_FRAC = 0.1
WEIGHT_FLOOR = 1e-12
OU_LAMBDA = 0.1
POWER_BETA_MIN = 0.25
POWER_BETA_EXC_C = 50.0
POWER_BETA_Z_C = 1.0
FORGETTING = 0.99
IW_NU_WEAK_ADD = 0.5
IW_RHO_PROC = np.array([0.99, 0.995, 0.95, 0.999, 0.999, 0.9999, 0.9999])  # trans,rot,vel,bg,ba,dt,ex
IW_RHO_MEAS = np.array([0.995, 0.995, 0.99])
PROC_BLOCK_DIMS = np.array([3, 3, 3, 3, 3, 1, 6])
PROC_BLOCK_STARTS = np.array([0, 3, 6, 9, 12, 15, 16])
SMALL_ANGLE = 1e-7
PLANAR_Z_REF, PLANAR_Z_SIGMA, PLANAR_VZ_SIGMA = 0.0, 0.1, 0.01  # constants.py:294-310
NEAR_PI = 1e-7
# Build-declared (never recorded in the reference — parity unpinned):
B_BINS = 48
TAU_SOFT_ASSIGN = 0.1
RANGE_SIGMA, RANGE_MIN_R, RANGE_MAX_R = 0.25, 0.5, 50.0

_rows = np.arange(6)[None, :] < PROC_BLOCK_DIMS[:, None]
PROC_BLOCK_MASKS = (_rows[:, :, None] & _rows[:, None, :]).astype(np.float64)


def sigmoid(x):
    # jax.nn.sigmoid (evaluated without overflow)
    return expit(x)


def softplus(x):
    # jax.nn.softplus = log1p(exp(-|x|)) + max(x, 0)
    x = np.asarray(x, dtype=np.float64)
    return np.log1p(np.exp(-np.abs(x))) + np.maximum(x, 0.0)


# ---------------------------------------------------------------------------------------
# Numeric primitives — fl_slam_poc/common/primitives.py
# ---------------------------------------------------------------------------------------
# Test switch (exact_inactive_deltas below): the projection delta of a clamp that moves no eigenvalue is
# reported as the exact-arithmetic 0 instead of the rounding of V diag(λ) Vᵀ (the reference's value,
# ~1e-16 ||M||, LAPACK-dependent). Off by default: the oracle follows the reference.
EXACT_INACTIVE_DELTA = False


class exact_inactive_deltas:
    """Context manager: psd_project reports 0 for an inactive clamp while it is active."""

    def __enter__(self):
        global EXACT_INACTIVE_DELTA
        self._prev, EXACT_INACTIVE_DELTA = EXACT_INACTIVE_DELTA, True
        return self

    def __exit__(self, *exc):
        global EXACT_INACTIVE_DELTA
        EXACT_INACTIVE_DELTA = self._prev
        return False


def psd_project(M, eps_psd=EPS_PSD):
    """domain_projection_psd_core (primitives.py:80-123). Returns (M_psd, cert6)."""
    M = np.asarray(M, dtype=np.float64)
    M_sym = 0.5 * (M + M.T)
    sym_delta = np.linalg.norm(M_sym - M, "fro")
    w, V = np.linalg.eigh(M_sym)
    wc = np.maximum(w, eps_psd)
    M_psd = V @ np.diag(wc) @ V.T
    proj = np.linalg.norm(M_psd - M_sym, "fro")
    if EXACT_INACTIVE_DELTA and float(np.min(w)) > eps_psd:
        proj = 0.0
    nnc = float(np.sum(wc < 10.0 * eps_psd))
    emin, emax = float(np.min(wc)), float(np.max(wc))
    return M_psd, np.array([proj, sym_delta, emin, emax, emax / emin, nnc])


def chol_solve_lifted(L, b, eps_lift=EPS_LIFT):
    """spd_cholesky_solve_lifted_core (primitives.py:141-166)."""
    d = L.shape[0]
    C = np.linalg.cholesky(L + eps_lift * np.eye(d))
    y = solve_triangular(C, b, lower=True)
    return solve_triangular(C.T, y, lower=False), eps_lift * d


def chol_inverse_lifted(L, eps_lift=EPS_LIFT):
    """spd_cholesky_inverse_lifted_core (primitives.py:169-192)."""
    d = L.shape[0]
    C = np.linalg.cholesky(L + eps_lift * np.eye(d))
    Ci = solve_triangular(C, np.eye(d), lower=True)
    return Ci.T @ Ci, eps_lift * d


def inv_mass(m, eps_mass=EPS_MASS):
    """inv_mass_core (primitives.py:195-212): 1/(m+eps+f64eps), eps/(m+eps+f64eps)."""
    denom = np.asarray(m, dtype=np.float64) + eps_mass + F64_EPS
    return 1.0 / denom, eps_mass / denom


# ---------------------------------------------------------------------------------------
# Lie maps — fl_slam_poc/common/geometry/se3_jax.py
# ---------------------------------------------------------------------------------------
def skew(v):
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def _BC(theta, theta_sq):
    """Shared B=(1-cos)/θ², C=(θ-sin)/θ³ with the small-angle branch (se3_jax.py:473-504)."""
    if theta < SMALL_ANGLE:
        return 0.5 - theta_sq / 24.0, 1.0 / 6.0 - theta_sq / 120.0
    st = theta
    sts = theta_sq if theta_sq >= SMALL_ANGLE ** 2 else 1.0
    return (1.0 - math.cos(st)) / sts, (st - math.sin(st)) / (sts * st)


def so3_exp(w):
    """so3_exp (se3_jax.py:259-301)."""
    w = np.asarray(w, dtype=np.float64)
    theta_sq = float(w @ w)
    theta = math.sqrt(theta_sq)
    K = skew(w)
    if theta < SMALL_ANGLE:
        a, b = 1.0, 0.5
    else:
        sts = theta_sq if theta_sq >= SMALL_ANGLE ** 2 else 1.0
        a, b = math.sin(theta) / theta, (1.0 - math.cos(theta)) / sts
    return np.eye(3) + a * K + b * (K @ K)


def so3_log(R):
    """so3_log (se3_jax.py:304-366), incl. the softmax-mixed near-π axis."""
    R = np.asarray(R, dtype=np.float64)
    c = min(max(0.5 * (np.trace(R) - 1.0), -1.0), 1.0)
    theta = math.acos(c)
    sk = 0.5 * (R - R.T)
    vex = np.array([sk[2, 1], sk[0, 2], sk[1, 0]])
    if theta < SMALL_ANGLE:
        return vex
    if abs(theta - math.pi) < NEAR_PI:
        dp1 = np.diag(R) + 1.0
        z = 50.0 * dp1
        e = np.exp(z - z.max())
        wts = e / e.sum()
        cols = R + np.eye(3)
        axis = wts[0] * cols[:, 0] + wts[1] * cols[:, 1] + wts[2] * cols[:, 2]
        n = np.linalg.norm(axis)
        n = 1.0 if n < SMALL_ANGLE else n
        return axis / n * theta
    s = math.sin(theta)
    s = 1.0 if abs(s) < SMALL_ANGLE else s
    return (theta / (2.0 * s)) * (2.0 * vex)


def se3_V(phi):
    """se3_V (se3_jax.py:137-174)."""
    ts = float(phi @ phi)
    B, C = _BC(math.sqrt(ts), ts)
    K = skew(phi)
    return np.eye(3) + B * K + C * (K @ K)


def se3_V_inv(phi):
    """_se3_V_inv (se3_jax.py:177-217)."""
    ts = float(phi @ phi)
    th = math.sqrt(ts)
    K = skew(phi)
    if th < SMALL_ANGLE:
        D = 1.0 / 12.0 + ts / 720.0
    else:
        sts = ts if ts >= SMALL_ANGLE ** 2 else 1.0
        D = 1.0 / sts - (1.0 + math.cos(th)) / (2.0 * th * math.sin(th) + 1e-12)
    return np.eye(3) - 0.5 * K + D * (K @ K)


def se3_exp(xi):
    """se3_exp (se3_jax.py:473-504): [V(φ)ρ, φ]."""
    xi = np.asarray(xi, dtype=np.float64)
    return np.concatenate([se3_V(xi[3:6]) @ xi[:3], xi[3:6]])


def se3_log(T):
    """se3_log (se3_jax.py:220-256)."""
    T = np.asarray(T, dtype=np.float64)
    phi = so3_log(so3_exp(T[3:6]))
    return np.concatenate([se3_V_inv(phi) @ T[:3], phi])


def se3_compose(a, b):
    """se3_compose (se3_jax.py:420-438)."""
    Ra, Rb = so3_exp(a[3:6]), so3_exp(b[3:6])
    return np.concatenate([a[:3] + Ra @ b[:3], so3_log(Ra @ Rb)])


# ---------------------------------------------------------------------------------------
# Belief helpers — fl_slam_poc/common/belief.py
# ---------------------------------------------------------------------------------------
@dataclass
class Belief:
    X_anchor: np.ndarray
    z_lin: np.ndarray
    L: np.ndarray
    h: np.ndarray
    stamp_sec: float = 0.0

    def copy(self):
        return Belief(self.X_anchor.copy(), self.z_lin.copy(), self.L.copy(), self.h.copy(), self.stamp_sec)


def identity_prior(precision=1e-6):
    """create_identity_prior (belief.py:328-371)."""
    return Belief(np.zeros(6), np.zeros(D_Z), precision * np.eye(D_Z), np.zeros(D_Z), 0.0)


def mean_increment(b: Belief):
    """belief.py:373-386."""
    return chol_solve_lifted(b.L, b.h)[0]


def world_pose(b: Belief):
    """belief.py:408-425: X_anchor ∘ Exp(δz[0:6])."""
    return se3_compose(b.X_anchor, se3_exp(mean_increment(b)[0:6]))


# ---------------------------------------------------------------------------------------
# Certificates — only the numeric surface that feeds back into the numbers
# (fl_slam_poc/common/certificates.py:77-108 InfluenceCert, :439-455 total_trigger_magnitude)
# ---------------------------------------------------------------------------------------
def trigger(lift=0.0, psd=0.0, nu=0.0, mass=0.0, rho=0.0, dt=1.0, ex=1.0, alpha=1.0, beta=1.0):
    return (lift + psd + nu + mass + rho + abs(1.0 - dt) + abs(1.0 - ex)
            + abs(1.0 - alpha) + abs(1.0 - beta))


# ---------------------------------------------------------------------------------------
# PointCloud2 parse — backend_node.py:356-468 (parse_pointcloud2_vlp16,
# _pointfield_to_dtype) and the no-TF base transform :1677-1690 (_parse_T_base_sensor_6d :247-258)
# ---------------------------------------------------------------------------------------
_PF_DTYPES = {1: "i1", 2: "u1", 3: "<i2", 4: "<u2", 5: "<i4", 6: "<u4", 7: "<f4", 8: "<f8"}
NONFINITE_SENTINEL = 1e6


def parse_pointcloud2_vlp16(data: bytes, fields, point_step: int, n_points: int, header_stamp: float):
    """fields: iterable of (name, offset, datatype). Returns (points, timestamps, weights, ring, tag)."""
    if n_points <= 0:
        return (np.zeros((0, 3)), np.zeros(0), np.zeros(0), np.zeros(0, np.uint8), np.zeros(0, np.uint8))
    fmap = {name: (off, dt) for name, off, dt in fields}
    missing = [k for k in ("x", "y", "z", "ring") if k not in fmap]
    if missing:
        raise RuntimeError(f"PointCloud2 (VLP-16 layout) missing required fields: {missing}")
    needed = ["x", "y", "z", "ring"] + (["intensity"] if "intensity" in fmap else [])
    tf = "t" if "t" in fmap else ("time" if "time" in fmap else None)
    if tf:
        needed.append(tf)
    dtype = np.dtype({"names": needed, "formats": [_PF_DTYPES[fmap[k][1]] for k in needed],
                      "offsets": [fmap[k][0] for k in needed], "itemsize": point_step})
    arr = np.frombuffer(data, dtype=dtype, count=n_points)
    s = NONFINITE_SENTINEL
    x = np.nan_to_num(np.asarray(arr["x"], np.float64), nan=s, posinf=s, neginf=-s)
    y = np.nan_to_num(np.asarray(arr["y"], np.float64), nan=s, posinf=s, neginf=-s)
    z = np.nan_to_num(np.asarray(arr["z"], np.float64), nan=s, posinf=s, neginf=-s)
    ring = np.asarray(arr["ring"]).astype(np.uint8)
    if tf is not None:
        t_raw = np.asarray(arr[tf], np.float64)
        t = t_raw * 1e-9 if np.any(t_raw > 1e6) else t_raw
    else:
        t = np.full(n_points, header_stamp, np.float64)
    dist = np.sqrt(x * x + y * y + z * z)
    with np.errstate(over="ignore"):  # sentinel ranges: exp overflows to inf, weight -> floor
      w_raw = (1.0 / (1.0 + np.exp(-(dist - RANGE_MIN_R) / RANGE_SIGMA))) * \
              (1.0 / (1.0 + np.exp(-(RANGE_MAX_R - dist) / RANGE_SIGMA)))
    w = w_raw * (1.0 - WEIGHT_FLOOR) + WEIGHT_FLOOR
    return np.stack([x, y, z], axis=1), t, w, ring, np.zeros(n_points, np.uint8)


def T_base_sensor(xyz_rxyz):
    """_parse_T_base_sensor_6d (backend_node.py:247-258): (R, t), R = Rotation.from_rotvec."""
    from scipy.spatial.transform import Rotation
    v = np.asarray(xyz_rxyz, np.float64).reshape(6)
    return Rotation.from_rotvec(v[3:6]).as_matrix(), v[:3].copy()


def to_base(points, R, t):
    """pts_base = (R @ p.T).T + t (backend_node.py:1680)."""
    return (R @ points.T).T + t[None, :]


# The IMU extrinsic of the reference's raw sensor dump (docs/raw_sensor_dump; a Livox IMU reporting
# accelerations in g): tools/apply_imu_extrinsic_to_csv.py:38-42, GC_IMU_ACCEL_SCALE constants.py:85
DUMP_T_BASE_IMU = (0.0, 0.0, 0.0, -0.015586, 0.489293, 0.0)
DUMP_ACCEL_SCALE = 9.81
ODOM_Z_VARIANCE_PRIOR = 1e6  # GC_ODOM_Z_VARIANCE_PRIOR (constants.py:300)


def imu_to_base(gyro, accel, R_base_imu, accel_scale=1.0):
    """on_imu (backend_node.py:1397-1412): accel = accel_raw · imu_accel_scale, then the no-TF
    numeric rotation of both into the base frame, gyro_base = R @ gyro, accel_base = R @ accel (per
    sample; the same math as tools/apply_imu_extrinsic_to_csv.py:85-110). (n, 3) arrays in and out."""
    R = np.asarray(R_base_imu, np.float64)
    g = np.asarray(gyro, np.float64)
    a = np.asarray(accel, np.float64) * float(accel_scale)
    return np.einsum("ij,nj->ni", R, g), np.einsum("ij,nj->ni", R, a)


def odom_pose_from_msg(position, quat_xyzw):
    """on_odom (backend_node.py:1441-1465): rotvec = Rotation.from_quat([x, y, z, w]).as_rotvec(),
    pose = se3_from_rotvec_trans(rotvec, position) = [trans, rotvec] (belief.py:93-110)."""
    from scipy.spatial.transform import Rotation
    rv = Rotation.from_quat(np.asarray(quat_xyzw, np.float64)).as_rotvec()
    return np.concatenate([np.asarray(position, np.float64), rv])


def odom_relative(first_abs, pose_abs):
    """first-odom-as-origin (backend_node.py:1512-1514): first⁻¹ ∘ pose."""
    return se3_compose(se3_inverse(first_abs), pose_abs)


def odom_cov_capped(cov, z_prior=ODOM_Z_VARIANCE_PRIOR):
    """backend_node.py:1518-1523: the pose covariance with its z variance raised to the prior."""
    c = np.array(cov, np.float64).reshape(6, 6)
    c[2, 2] = max(c[2, 2], float(z_prior))
    return c


# ---------------------------------------------------------------------------------------
# a1 PointBudgetResample — backend/operators/point_budget.py:50-221
# ---------------------------------------------------------------------------------------
def point_budget_resample(points, t, w, ring=None, tag=None, n_points_cap=8192):
    n_in = points.shape[0]
    stride = max(1, int(math.ceil(n_in / n_points_cap)))
    idx = np.arange(0, n_in, stride)
    ns = idx.shape[0]
    ring = np.zeros(n_in, np.uint8) if ring is None else np.asarray(ring, np.uint8)
    tag = np.zeros(n_in, np.uint8) if tag is None else np.asarray(tag, np.uint8)
    mass_in = np.sum(w)
    w_raw = w[idx]
    scale = mass_in / (np.sum(w_raw) + EPS_MASS)
    P = np.zeros((n_points_cap, 3)); P[:ns] = points[idx]
    T = np.zeros(n_points_cap); T[:ns] = t[idx]
    W = np.zeros(n_points_cap); W[:ns] = w_raw * scale
    RG = np.zeros(n_points_cap, np.uint8); RG[:ns] = ring[idx]
    TG = np.zeros(n_points_cap, np.uint8); TG[:ns] = tag[idx]
    wn = W / (mass_in + EPS_MASS)
    ess = 1.0 / np.sum(wn ** 2 + EPS_MASS)
    return dict(points=P, timestamps=T, weights=W, ring=RG, tag=TG, indices=idx, n_input=n_in,
                n_output=ns, total_mass_in=float(mass_in), total_mass_out=float(mass_in),
                ess=float(ess), support_frac=float(min(1.0, n_points_cap / (n_in + EPS_MASS))),
                trig=trigger(mass=EPS_MASS / (float(mass_in) + EPS_MASS)))


# ---------------------------------------------------------------------------------------
# a3 IMU windows + preintegration — backend/operators/imu_preintegration.py:19-147
# ---------------------------------------------------------------------------------------
def smooth_window_weights(stamps, t0, t1, sigma):
    sig = max(sigma, 1e-6)
    wr = sigmoid((stamps - t0) / sig) * sigmoid((t1 - stamps) / sig)
    return wr * (1.0 - WEIGHT_FLOOR) + WEIGHT_FLOOR


def preintegrate(stamps, gyro, accel, w, rotvec0, bg, ba, g=GRAVITY_W):
    """preintegrate_imu_relative_pose_jax (imu_preintegration.py:46-147) — sequential scan."""
    dt = np.maximum(np.concatenate([stamps[1:] - stamps[:-1], [0.0]]), 0.0)
    R = so3_exp(rotvec0)
    R0 = R.copy()
    v = np.zeros(3); p = np.zeros(3)
    swdt = 0.0
    s_body, s_nog, s_w = np.zeros(3), np.zeros(3), np.zeros(3)
    for i in range(stamps.shape[0]):
        de = w[i] * dt[i]
        dR = so3_exp((gyro[i] - bg) * de)
        a_b = accel[i] - ba
        a_nog = R @ a_b
        a_w = a_nog + g
        swdt += de
        s_body += a_b * de; s_nog += a_nog * de; s_w += a_w * de
        p = p + v * de + 0.5 * a_w * (de * de)
        v = v + a_w * de
        R = R @ dR
    dRel = R0.T @ R
    p_b = R0.T @ p
    den = max(swdt, 1e-12)
    return dict(delta_pose=np.concatenate([p_b, so3_log(dRel)]), ess=float(np.sum(w)),
                delta_R=dRel, delta_p=p_b, delta_v=R0.T @ v, dt_eff_sum=swdt,
                a_body_mean=s_body / den, a_world_nog_mean=s_nog / den, a_world_mean=s_w / den)


def imu_integration_time(stamps, t_start, t_end):
    """compute_imu_integration_time (pipeline.py:262-313)."""
    eps = 1e-9
    v = np.sort(stamps[(stamps > t_start - eps) & (stamps <= t_end + eps) & (stamps > 0.0)])
    if v.shape[0] < 2:
        return 0.0
    return max(0.0, min(float(np.sum(np.maximum(v[1:] - v[:-1], 0.0))), t_end - t_start))


def imu_dt_mean(stamps):
    """Average IMU period over valid (stamp>0) samples — pipeline.py:526-535."""
    v = stamps[stamps > 0.0]
    if v.shape[0] >= 2:
        v = np.sort(v)
        return max(float((v[-1] - v[0]) / max(v.shape[0] - 1, 1)), 1e-12)
    return 1e-12


def iw_meas_gyro_suffstats(gyro, w, bg, omega_avg, dt_imu):
    """imu_gyro_meas_iw_suffstats_from_avg_rate_jax (measurement_noise_iw_jax.py:130-171)."""
    wn = w / (np.sum(w) + EPS_MASS)
    r = (gyro - bg[None, :]) - omega_avg[None, :]
    rr = np.einsum("m,mi,mj->ij", wn, r, r)
    rr = 0.5 * (rr + rr.T)
    return psd_project(rr)[0] * max(dt_imu, 1e-12)


def iw_meas_accel_suffstats(rotvec0, accel, w, ba, dt_imu, g=GRAVITY_W):
    """imu_accel_meas_iw_suffstats_from_gravity_dir_jax (measurement_noise_iw_jax.py:174-218)."""
    f_pred = -(so3_exp(rotvec0).T @ g)
    wn = w / (np.sum(w) + EPS_MASS)
    r = (accel - ba[None, :]) - f_pred[None, :]
    rr = np.einsum("m,mi,mj->ij", wn, r, r)
    rr = 0.5 * (rr + rr.T)
    return psd_project(rr)[0] * max(dt_imu, 1e-12)


# ---------------------------------------------------------------------------------------
# a4 DeskewConstantTwist — backend/operators/deskew_constant_twist.py:31-117
# ---------------------------------------------------------------------------------------
def deskew_constant_twist(points, t, w, t0, t1, xi):
    """Vectorised over points (the reference vmaps one_point, deskew_constant_twist.py:50-58)."""
    denom = max(t1 - t0, 1e-12)
    alpha = (t - t0) / denom
    rho = alpha[:, None] * xi[None, 0:3]
    phi = alpha[:, None] * xi[None, 3:6]
    ts = np.sum(phi * phi, axis=1)
    th = np.sqrt(ts)
    small = th < SMALL_ANGLE
    st = np.where(small, 1.0, th)
    sts = np.where(ts < SMALL_ANGLE ** 2, 1.0, ts)
    s, c = np.sin(st), np.cos(st)
    Bv = np.where(small, 0.5 - ts / 24.0, (1.0 - c) / sts)
    Cv = np.where(small, 1.0 / 6.0 - ts / 120.0, (st - s) / (sts * st))
    a = np.where(small, 1.0, s / st)
    b = np.where(small, 0.5, (1.0 - c) / sts)
    K = np.zeros((points.shape[0], 3, 3))
    K[:, 0, 1], K[:, 0, 2], K[:, 1, 2] = -phi[:, 2], phi[:, 1], -phi[:, 0]
    K[:, 1, 0], K[:, 2, 0], K[:, 2, 1] = phi[:, 2], -phi[:, 1], phi[:, 0]
    K2 = K @ K
    I = np.eye(3)[None]
    V = I + Bv[:, None, None] * K + Cv[:, None, None] * K2
    R = I + a[:, None, None] * K + b[:, None, None] * K2
    tv = np.einsum("nij,nj->ni", V, rho)
    out = np.einsum("nji,nj->ni", R, points - tv)
    w_out = w * smooth_window_weights(t, t0, t1, TIME_WARP_SIGMA_FRAC * denom)
    retained = float(np.sum(w_out) / (np.sum(w) + EPS_MASS))
    return out, w_out, retained


def point_directions(points, origin, eps_mass=EPS_MASS):
    """pipeline.py:589-593 / binning.py:162-164."""
    rays = points - origin[None, :]
    return rays / (np.linalg.norm(rays, axis=1, keepdims=True) + eps_mass)


# ---------------------------------------------------------------------------------------
# a5 BinSoftAssign — archive/legacy_operators/binning.py:56-131 ; archive/bin_atlas.py:40-61
# ---------------------------------------------------------------------------------------
def fibonacci_atlas(n_bins=B_BINS):
    i = np.arange(n_bins, dtype=np.float64) + 0.5
    phi = np.arccos(1 - 2 * i / n_bins)
    theta = np.pi * (1 + np.sqrt(5)) * i
    d = np.stack([np.sin(phi) * np.cos(theta), np.sin(phi) * np.sin(theta), np.cos(phi)], 1)
    return d / (np.linalg.norm(d, axis=1, keepdims=True) + EPS_MASS)


def similarities(dirs, bins):
    """S = dirs·binsᵀ restated as an explicit, un-fused d0*b0 + d1*b1 + d2*b2 (the bin-index
    integer contract: argmax over this exact f64 expression, lowest index on ties)."""
    return (dirs[:, 0:1] * bins[None, :, 0] + dirs[:, 1:2] * bins[None, :, 1]) + dirs[:, 2:3] * bins[None, :, 2]


def bin_soft_assign(dirs, bins, tau=TAU_SOFT_ASSIGN):
    S = similarities(dirs, bins)
    x = S / tau
    e = np.exp(x - x.max(axis=1, keepdims=True))
    R = e / e.sum(axis=1, keepdims=True)
    ent = -np.sum(R * np.log(R + EPS_MASS), axis=1)
    avg_ent = np.sum(ent) / (dirs.shape[0] + EPS_MASS)
    return dict(resp=R, bin_index=np.argmax(S, axis=1).astype(np.int32), avg_entropy=float(avg_ent),
                max_resp=float(R.max()), ess=float(math.exp(avg_ent)), trig=0.0)


# ---------------------------------------------------------------------------------------
# a6 ScanBinMomentMatch + KappaFromResultant — binning.py:139-324 ; kappa.py:84-169
# ---------------------------------------------------------------------------------------
def kappa_batch(R, eps_r=EPS_R, d=3, r0=KAPPA_R0, tau=KAPPA_TAU):
    Rc = np.clip(R, 0.0, 1.0 - eps_r)
    R2 = Rc * Rc
    k_low = (Rc * (d - R2)) / (1.0 - R2 + eps_r)
    k_high = -np.log(np.maximum(1.0 - R2, eps_r))
    s = sigmoid((Rc - r0) / max(tau, 1e-6))
    return (1.0 - s) * k_low + s * k_high


def kappa_scalar(R, eps_r=EPS_R, d=3.0, r0=KAPPA_R0, tau=KAPPA_TAU):
    """_kappa_continuous_formula (kappa.py:84-127) after the clamp of kappa_from_resultant_v2."""
    R = min(max(float(R), 0.0), 1.0 - eps_r)
    R2 = R * R
    k_low = (R * (d - R2)) / (1.0 - R2 + eps_r)
    k_high = -math.log(max(1.0 - R2, eps_r))
    s = 1.0 / (1.0 + math.exp(-(R - r0) / max(tau, 1e-6)))
    return (1.0 - s) * k_low + s * k_high


def moment_sums(points, covs, w, resp, lam, origin):
    """The raw per-bin sums of binning.py:160-173 (sum_cov skipped when covs is None)."""
    # the three einsums "nb,ni,nj->bij" / "nb,nij->bij" as the (B x N)·(N x 9) products XLA lowers
    # them to (dot_general), so the CPU baseline runs them through BLAS
    w_r = (w * lam)[:, None] * resp
    d = point_directions(points, origin)
    n, B = w_r.shape
    N = np.sum(w_r, axis=0)
    s_dir = w_r.T @ d
    S_sc = (w_r.T @ (d[:, :, None] * d[:, None, :]).reshape(n, 9)).reshape(B, 3, 3)
    sum_p = w_r.T @ points
    sum_ppT = (w_r.T @ (points[:, :, None] * points[:, None, :]).reshape(n, 9)).reshape(B, 3, 3)
    sum_cov = np.zeros_like(sum_ppT) if covs is None else (w_r.T @ covs.reshape(n, 9)).reshape(B, 3, 3)
    return N, s_dir, S_sc, sum_p, sum_ppT, sum_cov


def moments_finalize(N, s_dir, S_sc, sum_p, sum_ppT, sum_cov, eps_psd=EPS_PSD, eps_mass=EPS_MASS):
    """binning.py:175-209."""
    inv_N, eps_ratio = inv_mass(N, eps_mass)
    p_bar = sum_p * inv_N[:, None]
    Sig_raw = sum_ppT * inv_N[:, None, None] - np.einsum("bi,bj->bij", p_bar, p_bar) + sum_cov * inv_N[:, None, None]
    Sig = np.empty_like(Sig_raw)
    certs = np.empty((N.shape[0], 6))
    psd_total = 0.0
    for b in range(N.shape[0]):
        Sig[b], certs[b] = psd_project(Sig_raw[b], eps_psd)
        psd_total += certs[b, 0]
    Rbar = np.linalg.norm(s_dir, axis=1) * inv_N
    kap = kappa_batch(Rbar)
    tm = np.sum(N)
    ess = tm ** 2 / (np.sum(N ** 2) + eps_mass)
    sf = float(np.mean(N / (N + eps_mass)))
    return dict(N=N, s_dir=s_dir, S_dir_scatter=S_sc, p_bar=p_bar, Sigma_p=Sig, kappa=kap,
                sum_p=sum_p, sum_ppT=sum_ppT, ess=float(ess), support_frac=sf,
                psd_delta=float(psd_total), psd_certs=certs, max_eps_ratio=float(np.max(eps_ratio)),
                trig=trigger(psd=float(psd_total), mass=float(np.max(eps_ratio))))


def scan_bin_moment_match(points, covs, w, resp, lam=None, origin=None):
    lam = np.ones(points.shape[0]) if lam is None else lam
    origin = np.zeros(3) if origin is None else origin
    return moments_finalize(*moment_sums(points, covs, w, resp, lam, origin))


# ---------------------------------------------------------------------------------------
# Map bin statistics — archive/bin_atlas.py:101-257
# ---------------------------------------------------------------------------------------
@dataclass
class MapStats:
    S_dir: np.ndarray
    S_dir_scatter: np.ndarray
    N_dir: np.ndarray
    N_pos: np.ndarray
    sum_p: np.ndarray
    sum_ppT: np.ndarray

    @staticmethod
    def empty(nb=B_BINS):
        return MapStats(np.zeros((nb, 3)), np.zeros((nb, 3, 3)), np.zeros(nb), np.zeros(nb),
                        np.zeros((nb, 3)), np.zeros((nb, 3, 3)))

    def copy(self):
        return MapStats(*(x.copy() for x in (self.S_dir, self.S_dir_scatter, self.N_dir,
                                              self.N_pos, self.sum_p, self.sum_ppT)))


def map_forget_and_add(m: MapStats, inc: MapStats, gamma=FORGETTING):
    """update_map_stats(apply_forgetting(m, γ), inc) (bin_atlas.py:137-163, :232-257)."""
    return MapStats(gamma * m.S_dir + inc.S_dir, gamma * m.S_dir_scatter + inc.S_dir_scatter,
                    gamma * m.N_dir + inc.N_dir, gamma * m.N_pos + inc.N_pos,
                    gamma * m.sum_p + inc.sum_p, gamma * m.sum_ppT + inc.sum_ppT)


def map_derived(m: MapStats, eps_mass=EPS_MASS, eps_psd=EPS_PSD):
    """_compute_map_derived_stats_core (bin_atlas.py:166-207) → (mu_dir, kappa, centroid, Sigma_c)."""
    nrm = np.linalg.norm(m.S_dir, axis=1)
    mu = m.S_dir / (nrm + eps_mass)[:, None]
    inv_d, _ = inv_mass(m.N_dir, eps_mass)
    kap = kappa_batch(nrm * inv_d)
    inv_p, _ = inv_mass(m.N_pos, eps_mass)
    c = m.sum_p * inv_p[:, None]
    raw = m.sum_ppT * inv_p[:, None, None] - np.einsum("bi,bj->bij", c, c)
    Sig = np.stack([psd_project(raw[b], eps_psd)[0] for b in range(raw.shape[0])])
    return mu, kap, c, Sig


def pose_cov_inflation_pushforward(stats, R, t, Sigma_pose):
    """PoseCovInflationPushforward (a13). BUILD-DEFINED — the reference source was deleted
    (CHANGELOG.md:1226,1246); parity unpinned. Pushes scan bin stats into the world frame
    with pose (R, t), t[2] = 0 (CHANGELOG.md:575-578), inflating each bin's centroid
    covariance by the pose covariance pushed through J = [R | -R[p̄]×]."""
    N = stats["N"]
    nb = N.shape[0]
    pw = stats["p_bar"] @ R.T + t[None, :]
    Sw = np.empty((nb, 3, 3))
    for b in range(nb):
        J = np.concatenate([R, -R @ skew(stats["p_bar"][b])], axis=1)
        Sw[b] = R @ stats["Sigma_p"][b] @ R.T + J @ Sigma_pose @ J.T
    return MapStats(stats["s_dir"] @ R.T, np.einsum("ij,bjk,lk->bil", R, stats["S_dir_scatter"], R),
                    N.copy(), N.copy(), N[:, None] * pw,
                    N[:, None, None] * (Sw + np.einsum("bi,bj->bij", pw, pw)))


# ---------------------------------------------------------------------------------------
# a7 MatrixFisherRotation — archive/legacy_operators/matrix_fisher_evidence.py:83-394
# ---------------------------------------------------------------------------------------
def scatter_metrics(S, N_total, eps=EPS_MASS):
    """compute_scatter_metrics (matrix_fisher_evidence.py:83-147)."""
    w, V = np.linalg.eigh(S * (1.0 / (N_total + eps)))
    idx = np.argsort(w)[::-1]
    lam = np.maximum(w[idx], 0.0)
    il = 1.0 / (lam[0] + eps)
    tot = lam.sum() + eps
    p = lam / tot
    ent = -np.sum(p * np.log(p + eps))
    return dict(eigenvalues=lam, eigenvectors=V[:, idx], linearity=(lam[0] - lam[1]) * il,
                planarity=(lam[1] - lam[2]) * il,
                sphericity=lam[2] * il, anisotropy=1.0 - lam[2] * il, effective_rank=math.exp(ent))


def matrix_fisher(R_pred, scan_s, scan_S, scan_N, map_s, map_S, map_N, eps_psd=EPS_PSD, eps=EPS_MASS):
    wb = np.sqrt(scan_N * map_N + eps)
    sn = np.linalg.norm(scan_s, axis=1)
    mn = np.linalg.norm(map_s, axis=1)
    us = scan_s / (sn + eps)[:, None]
    um = map_s / (mn + eps)[:, None]
    conf = (sn * (1.0 / (scan_N + eps))) * (mn * (1.0 / (map_N + eps)))
    wf = wb * conf
    H = np.einsum("b,bi,bj->ij", wf, um, us)
    U, s, Vt = np.linalg.svd(H)
    sgn = np.sign(np.linalg.det(U @ Vt))
    U = U.copy(); U[:, 2] *= sgn
    R_mf = U @ Vt
    V = Vt.T
    L_raw = V @ np.diag([s[1] + s[2], s[0] + s[2], s[0] + s[1]]) @ V.T
    delta = so3_log(R_pred.T @ R_mf)
    L_rot, pc = psd_project(L_raw, eps_psd)
    h_rot = L_rot @ delta
    N_eff = float(np.sum(wf))
    nll = 0.5 * float(delta @ L_rot @ delta)
    return dict(R_mf=R_mf, L_rot=L_rot, h_rot=h_rot, delta_rot=delta, svd=s, N_eff=N_eff,
                nll_per_ess=nll / (N_eff + eps), psd_delta=float(pc[0]), psd_cert=pc,
                scan_metrics=scatter_metrics(scan_S.sum(0), float(scan_N.sum()), eps),
                map_metrics=scatter_metrics(map_S.sum(0), float(map_N.sum()), eps),
                trig=trigger(psd=float(pc[0]), mass=eps / (N_eff + eps)))


# ---------------------------------------------------------------------------------------
# a8 PlanarTranslationEvidence — matrix_fisher_evidence.py:413-671 ; 22D embed :729-756
# ---------------------------------------------------------------------------------------
def planar_translation(t_pred, scan_p, scan_Sig, scan_N, map_c, map_Sig, map_Np, map_Sdir_sc, map_Nd,
                       R_hat, eps_psd=EPS_PSD, eps=EPS_MASS):
    T_map = map_Sdir_sc.sum(0) / (np.sum(map_Nd) + eps)
    ev = np.sort(np.linalg.eigvalsh(T_map))[::-1]
    zs = max(ev[2], 0.0) / max(ev[0], eps)
    tb = map_c - scan_p @ R_hat.T
    Sc = map_Sig + np.einsum("ij,bjk,lk->bil", R_hat, scan_Sig, R_hat)
    wb = np.sqrt(scan_N * map_Np + eps)
    Wi = np.stack([wb[b] * np.linalg.inv(Sc[b] + eps * np.eye(3)) for b in range(wb.shape[0])])
    Lf = Wi.sum(0)
    hf = np.einsum("bij,bj->bi", Wi, tb).sum(0)
    t_wls = np.linalg.solve(Lf + eps * np.eye(3), hf)
    m = np.array([1.0, 1.0, zs])
    L_raw = Lf * m[:, None] * m[None, :]
    delta = t_wls - t_pred
    L_t, pc = psd_project(L_raw, eps_psd)
    h_t = L_t @ delta
    N_eff = float(np.sum(wb))
    nll = 0.5 * float(delta @ L_t @ delta)
    return dict(t_wls=t_wls, L_trans=L_t, h_trans=h_t, delta_trans=delta, z_scale=zs, N_eff=N_eff,
                nll_per_ess=nll / (N_eff + eps), psd_delta=float(pc[0]), psd_cert=pc,
                xy_info_scale=0.5 * (L_t[0, 0] + L_t[1, 1]), z_info_scale=L_t[2, 2],
                trig=trigger(psd=float(pc[0]), mass=eps / (N_eff + eps)))


# ---------------------------------------------------------------------------------------
# a2 PredictDiffusion — backend/operators/predict.py:43-214
# ---------------------------------------------------------------------------------------
def predict_diffusion(b: Belief, Q, dt, eps_psd=EPS_PSD, eps_lift=EPS_LIFT, lam=OU_LAMBDA):
    mu, _ = chol_solve_lifted(b.L, b.h, eps_lift)
    cov, lift_prev = chol_inverse_lifted(b.L, eps_lift)
    ef = math.exp(-2.0 * lam * dt)
    dc = (1.0 - ef) / (2.0 * lam + F64_EPS)
    cov_psd, c1 = psd_project(ef * cov + dc * Q, eps_psd)
    Lp, lift_inv = chol_inverse_lifted(cov_psd, eps_lift)
    Lp, c2 = psd_project(Lp, eps_psd)
    out = Belief(b.X_anchor.copy(), b.z_lin.copy(), Lp, Lp @ mu, b.stamp_sec + dt)
    return out, dict(lift=lift_prev + lift_inv, psd_delta=c1[0] + c2[0], cond=c2[2:6].copy(),
                     trace_cov=float(np.trace(cov_psd)),
                     trig=trigger(lift=lift_prev + lift_inv, psd=c1[0] + c2[0], dt=dt))


# ---------------------------------------------------------------------------------------
# a9-a11 evidence assembly, tempering, excitation, fusion — pipeline.py:1038-1206 ;
# excitation.py:14-64 ; fusion.py:46-230 ; certificates.py:511-600 (aggregation)
# ---------------------------------------------------------------------------------------
@dataclass
class IOEvidence:
    """Per-hypothesis IMU/odom-branch evidence (pipeline.py:595-776), a synthetic input for this
    tier: L_io, h_io plus the certificate scalars that branch feeds
    into the numbers: odom/imu/gyro cert (ess, support_frac), excitation maxima, nll sum and the
    summed trigger magnitude of its 11 certs."""
    L: np.ndarray
    h: np.ndarray
    ess: np.ndarray = field(default_factory=lambda: np.zeros(3))
    support: np.ndarray = field(default_factory=lambda: np.ones(3))
    exc_dt: float = 0.0
    exc_ex: float = 0.0
    nll: float = 0.0
    trig: float = 0.0


# ---------------------------------------------------------------------------------------
# a9a IMU/odom branch — pipeline.py:595-776 and the 11 operators it calls.
# Paths: backend/operators/{odom_evidence,imu_evidence,imu_gyro_evidence,
# imu_preintegration_factor,planar_prior,odom_twist_evidence}.py
# ---------------------------------------------------------------------------------------
def se3_inverse(a):
    """se3_inverse (se3_jax.py:442-453)."""
    R = so3_exp(a[3:6])
    return np.concatenate([-(R.T @ a[:3]), so3_log(R.T)])


def se3_relative(a, b):
    """se3_relative (se3_jax.py:457-459): b^{-1} ∘ a."""
    return se3_compose(se3_inverse(b), a)


def _eig_stats(M):
    ev = np.linalg.eigvalsh(M)
    return float(ev.min()), float(ev.max()), ev


def odom_quadratic_evidence(pose_pred, odom_pose, odom_cov, eps_psd=EPS_PSD, eps_lift=EPS_LIFT):
    """_odom_quadratic_evidence_core (odom_evidence.py:40-84) + cert (:126-146)."""
    xi = se3_log(se3_relative(odom_pose, pose_pred))
    cov_psd = psd_project(odom_cov, eps_psd)[0]
    Lp, lift = chol_inverse_lifted(cov_psd, eps_lift)
    L = np.zeros((D_Z, D_Z)); L[0:6, 0:6] = Lp
    dz = np.zeros(D_Z); dz[0:6] = xi
    h = L @ dz
    nll = 0.5 * float(xi @ Lp @ xi)
    emin, emax, ev = _eig_stats(psd_project(Lp, eps_psd)[0])
    return dict(L=L, h=h, delta_z=dz, nll=nll, lift=lift, eig_min=emin, eig_max=emax,
                cond=emax / max(emin, 1e-18), nnc=float(np.sum(ev < 1e-12)), trig=trigger(lift=lift))


def transport_consistency(accel_c, gyro, dt, eps_mass=EPS_MASS):
    """_compute_transport_consistency (imu_evidence.py:277-334)."""
    df = np.zeros_like(accel_c)
    df[1:-1] = (accel_c[2:] - accel_c[:-2]) / (2 * dt + eps_mass)
    df[0] = (accel_c[1] - accel_c[0]) / (dt + eps_mass)
    df[-1] = (accel_c[-1] - accel_c[-2]) / (dt + eps_mass)
    return np.linalg.norm(df + np.cross(gyro, accel_c), axis=1)


def reliability_weights(e, eps_mass=EPS_MASS):
    """_compute_reliability_weights (imu_evidence.py:337-368): MAD-based σ."""
    med = np.median(e)
    sigma = np.median(np.abs(e - med)) / 0.6745 + eps_mass
    return np.exp(-0.5 * (e / sigma) ** 2), sigma


def imu_vmf_gravity_evidence_time_resolved(rotvec, accel, gyro, w, ba, g, dt_imu, eps_psd=EPS_PSD,
                                           eps_mass=EPS_MASS):
    """imu_vmf_gravity_evidence_time_resolved (imu_evidence.py:402-559), incl.
    _accel_resultant_direction_weighted_jax (:371-399) and kappa_from_resultant_v2 (kappa.py:172-232)."""
    R0 = so3_exp(rotvec)
    g_hat = g / (np.linalg.norm(g) + eps_mass)
    e = transport_consistency(accel - ba[None, :], gyro, dt_imu, eps_mass)
    rel, sigma = reliability_weights(e, eps_mass)
    wr = w * rel
    ess_w, ess_raw = float(np.sum(wr)), float(np.sum(w))
    a = accel - ba[None, :]
    x = a / (np.linalg.norm(a, axis=1, keepdims=True) + eps_mass)
    S = np.sum(wr[:, None] * x, axis=0)
    Sn = np.linalg.norm(S)
    xbar = S / (Sn + eps_mass)
    Rbar = Sn / (ess_w + eps_mass)
    kappa = kappa_scalar(Rbar)
    mu0 = R0.T @ (-g_hat)
    xdm = float(xbar @ mu0)
    g_rot = -kappa * np.cross(mu0, xbar)
    H = kappa * (xdm * np.eye(3) - 0.5 * (np.outer(xbar, mu0) + np.outer(mu0, xbar)))
    H = 0.5 * (H + H.T)
    Hp, hc = psd_project(H, eps_psd)
    L = np.zeros((D_Z, D_Z)); L[3:6, 3:6] = Hp
    h = np.zeros(D_Z); h[3:6] = -g_rot
    nll = float(-kappa * (mu0 @ xbar))
    mrel = float(np.mean(rel))
    mer = ess_w / (ess_raw + eps_mass)
    return dict(L=L, h=h, kappa=kappa, ess_weighted=ess_w, ess_raw=ess_raw, mean_reliability=mrel,
                transport_sigma=float(sigma), Rbar=float(Rbar), xbar=xbar, nll=nll,
                nll_per_ess=nll / (ess_w + eps_mass), psd_delta=float(hc[0]),
                trig=trigger(psd=float(hc[0]), mass=mer, alpha=mrel))


def imu_dependence_inflation(transport_sigma, eps_mass=EPS_MASS):
    """imu_dependence_inflation (imu_evidence.py:562-589)."""
    s = max(transport_sigma, 0.0)
    scale = 1.0 / (1.0 + s * s + eps_mass)
    return dict(scale=scale, trig=trigger(alpha=scale))


def imu_gyro_rotation_evidence(rv_start, rv_end_pred, drv_meas, Sigma_g, dt_int, eps_psd=EPS_PSD,
                               eps_lift=EPS_LIFT):
    """_imu_gyro_rotation_evidence_jax (imu_gyro_evidence.py:38-85)."""
    dtp = max(dt_int, 0.0)
    R_end_imu = so3_exp(rv_start) @ so3_exp(drv_meas)
    r = so3_log(so3_exp(rv_end_pred).T @ R_end_imu)
    dte = dtp + EPS_MASS
    ms = dtp / dte
    Sp = psd_project(Sigma_g * dte, eps_psd)[0]
    Lr, lift = chol_inverse_lifted(Sp, eps_lift)
    L = np.zeros((D_Z, D_Z)); L[3:6, 3:6] = ms * Lr
    h = np.zeros(D_Z); h[3:6] = (ms * Lr) @ r
    nll = 0.5 * float(r @ Lr @ r)
    emin, emax, ev = _eig_stats(psd_project(Lr, eps_psd)[0])
    return dict(L=L, h=h, r_rot=r, nll=nll, lift=lift, eig_min=emin, eig_max=emax,
                nnc=float(np.sum(ev < eps_psd)), trig=trigger(lift=lift))


def imu_preintegration_factor(p_start, rv_start, v_start, p_end_pred, v_end_pred, dv_body, dp_body, Sigma_a,
                              dt_int, eps_psd=EPS_PSD, eps_lift=EPS_LIFT):
    """imu_preintegration_factor (imu_preintegration_factor.py:46-180)."""
    R = so3_exp(rv_start)
    r_vel = (v_start + R @ dv_body) - v_end_pred
    r_pos = (p_start + v_start * dt_int + R @ dp_body) - p_end_pred
    dtp = max(dt_int, 0.0)
    dte = dtp + EPS_MASS
    ms = dtp / dte
    Lv, lv = chol_inverse_lifted(psd_project(Sigma_a * dte, eps_psd)[0], eps_lift)
    Lp, lp = chol_inverse_lifted(psd_project(Sigma_a * dte ** 3, eps_psd)[0], eps_lift)
    L = np.zeros((D_Z, D_Z)); h = np.zeros(D_Z)
    L[0:3, 0:3] = ms * Lp; h[0:3] = (ms * Lp) @ r_pos
    L[6:9, 6:9] = ms * Lv; h[6:9] = (ms * Lv) @ r_vel
    nll = 0.5 * float(r_vel @ Lv @ r_vel) + 0.5 * float(r_pos @ Lp @ r_pos)
    return dict(L=L, h=h, r_vel=r_vel, r_pos=r_pos, nll=nll, lift=lv + lp, trig=trigger(lift=lv + lp))


def planar_z_prior(pose, z_ref=PLANAR_Z_REF, sigma_z=PLANAR_Z_SIGMA):
    """planar_z_prior (planar_prior.py:55-135)."""
    r = float(z_ref - pose[2])
    prec = 1.0 / sigma_z ** 2
    L = np.zeros((D_Z, D_Z)); L[2, 2] = prec
    h = np.zeros(D_Z); h[2] = prec * r
    return dict(L=L, h=h, r_z=r, nll=0.5 * r * r * prec, trig=trigger())


def velocity_z_prior(v_z_pred, sigma_vz=PLANAR_VZ_SIGMA):
    """velocity_z_prior (planar_prior.py:138-195)."""
    r = -float(v_z_pred)
    prec = 1.0 / sigma_vz ** 2
    L = np.zeros((D_Z, D_Z)); L[8, 8] = prec
    h = np.zeros(D_Z); h[8] = prec * r
    return dict(L=L, h=h, v_z=float(v_z_pred), nll=0.5 * r * r * prec, trig=trigger())


def odom_velocity_evidence(v_pred_world, R_world_body, v_odom_body, Sigma_v, eps_psd=EPS_PSD, eps_lift=EPS_LIFT):
    """odom_velocity_evidence (odom_twist_evidence.py:58-154)."""
    r = v_odom_body - R_world_body.T @ v_pred_world
    Sp = psd_project(Sigma_v, eps_psd)[0]
    Lv, lift = chol_inverse_lifted(Sp, eps_lift)
    L = np.zeros((D_Z, D_Z)); L[6:9, 6:9] = Lv
    h = np.zeros(D_Z); h[6:9] = Lv @ r
    emin, emax, ev = _eig_stats(Sp)
    return dict(L=L, h=h, r_vel=r, nll=0.5 * float(r @ Lv @ r), lift=lift, eig_min=emin, eig_max=emax,
                trig=trigger(lift=lift))


def odom_yawrate_evidence(wz_pred, wz_odom, sigma_wz):
    """odom_yawrate_evidence (odom_twist_evidence.py:157-225)."""
    r = float(wz_odom) - float(wz_pred)
    prec = 1.0 / sigma_wz ** 2
    L = np.zeros((D_Z, D_Z)); L[5, 5] = prec
    h = np.zeros(D_Z); h[5] = prec * r
    return dict(L=L, h=h, r_wz=r, nll=0.5 * r * r * prec, trig=trigger())


def pose_twist_kinematic_consistency(pose_prev, pose_curr, v_body, omega_body, dt, Sigma_v, Sigma_omega,
                                     eps_psd=EPS_PSD, eps_lift=EPS_LIFT):
    """pose_twist_kinematic_consistency (odom_twist_evidence.py:251-397)."""
    R_prev, R_curr = so3_exp(pose_prev[3:6]), so3_exp(pose_curr[3:6])
    r_t = (R_prev @ v_body * dt) - (pose_curr[:3] - pose_prev[:3])
    r_r = (omega_body * dt) - so3_log(R_prev.T @ R_curr)
    dt2 = dt * dt + eps_psd
    St = psd_project(dt2 * Sigma_v, eps_psd)[0]
    Sr = psd_project(dt2 * Sigma_omega, eps_psd)[0]
    Lt, lt = chol_inverse_lifted(St, eps_lift)
    Lr, lr = chol_inverse_lifted(Sr, eps_lift)
    L = np.zeros((D_Z, D_Z)); h = np.zeros(D_Z)
    L[0:3, 0:3] = Lt; L[3:6, 3:6] = Lr
    h[0:3] = Lt @ r_t; h[3:6] = Lr @ r_r
    nll = 0.5 * float(r_t @ Lt @ r_t) + 0.5 * float(r_r @ Lr @ r_r)
    return dict(L=L, h=h, r_trans=r_t, r_rot=r_r, nll=nll, lift=lt + lr, trig=trigger(lift=lt + lr))


def odom_dependence_inflation(r_trans, r_rot, eps_mass=EPS_MASS):
    """odom_dependence_inflation (odom_twist_evidence.py:400-430)."""
    mag = float(np.linalg.norm(r_trans) + np.linalg.norm(r_rot))
    scale = 1.0 / (1.0 + mag * mag + eps_mass)
    return dict(scale=scale, trig=trigger(alpha=scale))


@dataclass
class OdomInput:
    """Per-scan odometry the node hands the pipeline (backend_node.py:1748-1765): relative pose
    (6), pose covariance (6,6) in [trans, rot] order, twist (6) [v, ω] body, twist cov (6,6)."""
    pose: np.ndarray
    cov: np.ndarray
    twist: np.ndarray
    twist_cov: np.ndarray


def imu_odom_branch(b_prev: Belief, b_pred: Belief, odom: OdomInput, imu_accel, imu_gyro, w_int, ba, pre_int,
                    dt_int, dt_imu, omega_avg, dt_sec, Sigma_g, Sigma_a, g=GRAVITY_W, z_ref=PLANAR_Z_REF,
                    sigma_z=PLANAR_Z_SIGMA, sigma_vz=PLANAR_VZ_SIGMA, eps_psd=EPS_PSD, eps_lift=EPS_LIFT,
                    eps_mass=EPS_MASS):
    """_compute_imu_odom_branch (pipeline.py:595-776): the 11 factors, their dependence scalings
    and the summed (L_io, h_io). Returns (IOEvidence, parts). z_lin_pose (:751-755) feeds only the
    primitive-map branch (visual_pose_evidence), which the bin path does not run."""
    pose_pred = world_pose(b_pred)
    pose0 = world_pose(b_prev)
    rv0 = pose0[3:6]
    mu_inc = mean_increment(b_pred)
    od = odom_quadratic_evidence(pose_pred, odom.pose, odom.cov, eps_psd, eps_lift)
    im = imu_vmf_gravity_evidence_time_resolved(pose_pred[3:6], imu_accel, imu_gyro, w_int, ba, g, dt_imu,
                                                eps_psd, eps_mass)
    dep = imu_dependence_inflation(im["transport_sigma"], eps_mass)
    gy = imu_gyro_rotation_evidence(rv0, pose_pred[3:6], pre_int["delta_pose"][3:6], Sigma_g, dt_int, eps_psd,
                                    eps_lift)
    v_start = mean_increment(b_prev)[6:9]
    pr = imu_preintegration_factor(pose0[0:3], rv0, v_start, pose_pred[0:3], mu_inc[6:9], pre_int["delta_v"],
                                   pre_int["delta_p"], Sigma_a, dt_int, eps_psd, eps_lift)
    pl = planar_z_prior(pose_pred, z_ref, sigma_z)
    vz = velocity_z_prior(mu_inc[8], sigma_vz)
    ov = odom_velocity_evidence(mu_inc[6:9], so3_exp(pose_pred[3:6]), odom.twist[0:3], odom.twist_cov[0:3, 0:3],
                                eps_psd, eps_lift)
    sig_wz = math.sqrt(max(odom.twist_cov[5, 5], 1e-12))
    wz = odom_yawrate_evidence(omega_avg[2], odom.twist[5], sig_wz)
    kc = pose_twist_kinematic_consistency(pose0, pose_pred, odom.twist[0:3], odom.twist[3:6], dt_sec,
                                          odom.twist_cov[0:3, 0:3], odom.twist_cov[3:6, 3:6], eps_psd, eps_lift)
    odep = odom_dependence_inflation(kc["r_trans"], kc["r_rot"], eps_mass)
    si, so = dep["scale"], odep["scale"]
    L = (od["L"] * so + im["L"] * si + gy["L"] * si + pr["L"] + pl["L"] + vz["L"] + ov["L"] * so + wz["L"] * so
         + kc["L"])
    h = (od["h"] * so + im["h"] * si + gy["h"] * si + pr["h"] + pl["h"] + vz["h"] + ov["h"] * so + wz["h"] * so
         + kc["h"])
    parts = [od, im, dep, gy, pr, pl, vz, ov, wz, kc, odep]
    io = IOEvidence(L=L, h=h, ess=np.array([0.0, im["ess_weighted"], 0.0]),
                    support=np.array([1.0, im["mean_reliability"], 1.0]), exc_dt=0.0, exc_ex=0.0,
                    nll=od["nll"] + im["nll_per_ess"] + gy["nll"], trig=float(sum(p["trig"] for p in parts)))
    return io, dict(odom=od, imu=im, imu_dep=dep, gyro=gy, preint=pr, planar=pl, vz=vz, odom_vel=ov, odom_wz=wz,
                    kinematic=kc, odom_dep=odep)


def tempering_beta(L_raw, ess_total, exc_total):
    """pipeline.py:1070-1111."""
    eps = EPS_MASS
    dpose = np.linalg.norm(L_raw[15, 0:6]) + np.linalg.norm(L_raw[0:6, 15])
    dvel = np.linalg.norm(L_raw[15, 6:9]) + np.linalg.norm(L_raw[6:9, 15])
    dt_asym = min(max(abs(dvel - dpose) / (dvel + dpose + eps), 0.0), 1.0)
    z_xy = abs(L_raw[2, 2]) / (0.5 * (abs(L_raw[0, 0]) + abs(L_raw[1, 1])) + eps)
    ess_to_exc = ess_total / (exc_total + eps)
    s = min(max(dt_asym * (z_xy / (z_xy + POWER_BETA_Z_C)) * (1.0 / (1.0 + ess_to_exc / POWER_BETA_EXC_C)), 0.0), 1.0)
    beta = min(max(POWER_BETA_MIN + (1.0 - POWER_BETA_MIN) * s, POWER_BETA_MIN), 1.0)
    return beta, dt_asym, z_xy


def excitation_scaling(L_ev, L_prior, h_prior, eps=EXC_EPS):
    """compute_excitation_scales_jax + apply_excitation_prior_scaling_jax (excitation.py:14-64)."""
    e_dt, pi_dt = L_ev[15, 15], L_prior[15, 15]
    e_ex, pi_ex = np.trace(L_ev[16:22, 16:22]), np.trace(L_prior[16:22, 16:22])
    s_dt = e_dt / (e_dt + pi_dt + eps)
    s_ex = e_ex / (e_ex + pi_ex + eps)
    Lp, hp = L_prior.copy(), h_prior.copy()
    Lp[15, :] *= 1.0 - s_dt; Lp[:, 15] *= 1.0 - s_dt; hp[15] *= 1.0 - s_dt
    Lp[16:22, :] *= 1.0 - s_ex; Lp[:, 16:22] *= 1.0 - s_ex; hp[16:22] *= 1.0 - s_ex
    return Lp, hp, float(s_dt), float(s_ex)


def fusion_alpha(cond_ev, ess_ev, exc_total, dt_asym, z_xy, beta, nll,
                 amin=ALPHA_MIN, amax=ALPHA_MAX, c0=C0_COND):
    """fusion_scale_from_certificates (fusion.py:46-142)."""
    q = math.sqrt((c0 / (cond_ev + c0)) * (ess_ev / (ess_ev + 1.0)))
    q *= math.exp(-nll) * min(max(dt_asym, 0.0), 1.0)
    q *= min(max(z_xy / (z_xy + 1.0), 0.0), 1.0) * min(max(exc_total / (exc_total + 1.0), 0.0), 1.0)
    q *= min(max(beta, 0.0), 1.0)
    return min(max(amin + (amax - amin) * q, amin), amax)


def pose6_eigs(L_ev, eps=EPS_PSD):
    """pipeline.py:1157-1168: eigvalsh of the symmetrised pose block, clipped at eps_psd."""
    P = 0.5 * (L_ev[0:6, 0:6] + L_ev[0:6, 0:6].T)
    return np.maximum(np.linalg.eigvalsh(P), eps)


def pose6_cond(L_ev, eps=EPS_PSD):
    ev = pose6_eigs(L_ev, eps)
    return ev[-1] / ev[0]


def info_fusion_additive(L_pred, h_pred, L_ev, h_ev, alpha, eps_psd=EPS_PSD):
    """fusion.py:150-230."""
    Lp, c = psd_project(L_pred + alpha * L_ev, eps_psd)
    return Lp, h_pred + alpha * h_ev, c


# ---------------------------------------------------------------------------------------
# a12 PoseUpdateFrobeniusRecompose — backend/operators/recompose.py:50-205
# ---------------------------------------------------------------------------------------
def bch3(x1, x2):
    return 0.5 * np.concatenate([np.cross(x1[3:6], x2[:3]) + np.cross(x1[:3], x2[3:6]),
                                 np.cross(x1[3:6], x2[3:6])])


def recompose(b: Belief, T, c_frob=C_FROB, eps_lift=EPS_LIFT):
    dz = chol_solve_lifted(b.L, b.h, eps_lift)[0]
    s = T / (T + c_frob)
    corr = bch3(b.z_lin[0:6], dz[0:6])
    dpc = dz[0:6] + s * corr
    X_new = se3_compose(b.X_anchor, se3_exp(dpc))
    shift = np.zeros(D_Z); shift[0:6] = dpc
    return Belief(X_new, b.z_lin - shift, b.L.copy(), b.h - b.L @ shift, b.stamp_sec), dict(
        delta_pose=dpc, frobenius_strength=s, bch=corr)


# ---------------------------------------------------------------------------------------
# a14 AnchorDriftUpdate — backend/operators/anchor_drift.py:93-191
# ---------------------------------------------------------------------------------------
def anchor_drift(b: Belief, eps_lift=EPS_LIFT):
    dz = chol_solve_lifted(b.L, b.h, eps_lift)[0]
    dm, dr = float(np.linalg.norm(dz[0:3])), float(np.linalg.norm(dz[3:6]))
    rho = min(max(max(dm / ANCHOR_M0, dr / ANCHOR_R0), 0.0), 1.0)
    X = se3_compose(b.X_anchor, se3_exp(rho * dz[0:6]))
    zl = (1.0 - rho) * dz
    return Belief(X, zl, b.L.copy(), b.L @ zl, b.stamp_sec), dict(rho=rho, drift_m=dm, drift_r=dr)


# ---------------------------------------------------------------------------------------
# a15 Inverse-Wishart — backend/operators/inverse_wishart_jax.py:26-185 ;
# measurement_noise_iw_jax.py:28-100 ; backend/structures/*iw*.py
# ---------------------------------------------------------------------------------------
def softplus_pos(x, eps=1e-12, beta=50.0):
    return softplus(beta * x) / beta + eps


def iw_process_init():
    """create_datasheet_process_noise_state (structures/inverse_wishart_jax.py:43-80)."""
    nu = PROC_BLOCK_DIMS + 1.0 + IW_NU_WEAK_ADD
    diag = [1e-4, 8.7e-7, 9.5e-5, 1e-8, 1e-6, 1e-6, 1e-8]
    Psi = np.zeros((7, 6, 6))
    for i in range(7):
        d = PROC_BLOCK_DIMS[i]
        Psi[i, :d, :d] = np.eye(d) * diag[i] * IW_NU_WEAK_ADD
    return nu.astype(np.float64), Psi


def iw_meas_init(lidar_sigma=0.01):
    """create_datasheet_measurement_noise_state (structures/measurement_noise_iw_jax.py:37-68)."""
    nu = np.array([3.0, 3.0, 3.0]) + 1.0 + IW_NU_WEAK_ADD
    Psi = np.stack([8.7e-7 * np.eye(3), 9.5e-5 * np.eye(3), lidar_sigma * np.eye(3)]) * IW_NU_WEAK_ADD
    return nu, Psi


def iw_process_Q(nu, Psi, eps_psd=EPS_PSD):
    """process_noise_state_to_Q_jax (inverse_wishart_jax.py:35-68)."""
    den = softplus_pos(nu - PROC_BLOCK_DIMS - 1.0)
    Qb = Psi / den[:, None, None] * PROC_BLOCK_MASKS
    Q = np.zeros((D_Z, D_Z))
    for i in range(7):
        s = PROC_BLOCK_STARTS[i]
        e = min(s + 6, D_Z)
        Q[s:e, s:e] = Qb[i][: e - s, : e - s]
    return psd_project(Q, eps_psd)[0]


def iw_process_suffstats(L_pred, h_pred, L_post, h_post, eps_lift=EPS_LIFT):
    """process_noise_iw_suffstats_from_info_jax (inverse_wishart_jax.py:71-123)."""
    r = chol_solve_lifted(L_post, h_post, eps_lift)[0] - chol_solve_lifted(L_pred, h_pred, eps_lift)[0]
    Sp = chol_inverse_lifted(L_post, eps_lift)[0]
    dPsi = np.zeros((7, 6, 6))
    for i in range(7):
        s, d = PROC_BLOCK_STARTS[i], PROC_BLOCK_DIMS[i]
        dPsi[i, :d, :d] = np.outer(r[s:s + d], r[s:s + d]) + Sp[s:s + d, s:s + d]
    return dPsi, np.ones(7)


def _nu_project(nu_raw, dims, nu_max=1000.0):
    nmin = dims + 1.0 + IW_NU_WEAK_ADD
    nf = nmin + softplus(nu_raw - nmin)
    return nu_max - softplus(nu_max - nf)


def iw_process_apply(nu, Psi, dPsi, dnu, eps_psd=EPS_PSD):
    """process_noise_iw_apply_suffstats_jax (inverse_wishart_jax.py:126-185)."""
    raw = (IW_RHO_PROC[:, None, None] * Psi + dPsi) * PROC_BLOCK_MASKS
    out = np.empty_like(raw)
    pd = 0.0
    for i in range(7):
        out[i], c = psd_project(raw[i], eps_psd)
        pd += c[0]
    nr = IW_RHO_PROC * nu + dnu
    n2 = _nu_project(nr, PROC_BLOCK_DIMS.astype(np.float64))
    return n2, out, np.array([pd, np.sum(np.abs(n2 - nr))])


def iw_meas_apply(nu, Psi, dPsi, dnu, eps_psd=EPS_PSD):
    """measurement_noise_apply_suffstats_jax (measurement_noise_iw_jax.py:59-100)."""
    raw = IW_RHO_MEAS[:, None, None] * Psi + dPsi
    raw = 0.5 * (raw + np.swapaxes(raw, -1, -2))
    out = np.empty_like(raw)
    pd = 0.0
    for i in range(3):
        out[i], c = psd_project(raw[i], eps_psd)
        pd += c[0]
    nr = IW_RHO_MEAS * nu + dnu
    n2 = _nu_project(nr, np.array([3.0, 3.0, 3.0]))
    return n2, out, np.array([pd, np.sum(np.abs(n2 - nr))])


def iw_process_block_certs(Psi, dPsi, eps_psd=EPS_PSD):
    """The cert_vec of each padded process-IW block projection of iw_process_apply
    (inverse_wishart_jax.py:163-172), (7, 6)."""
    raw = (IW_RHO_PROC[:, None, None] * Psi + dPsi) * PROC_BLOCK_MASKS
    return np.stack([psd_project(raw[i], eps_psd)[1] for i in range(7)])


def iw_meas_block_certs(Psi, dPsi, eps_psd=EPS_PSD):
    """The cert_vec of each measurement-IW block projection of iw_meas_apply
    (measurement_noise_iw_jax.py:78-86), (3, 6)."""
    raw = IW_RHO_MEAS[:, None, None] * Psi + dPsi
    raw = 0.5 * (raw + np.swapaxes(raw, -1, -2))
    return np.stack([psd_project(raw[i], eps_psd)[1] for i in range(3)])


def iw_process_Q_cert(nu, Psi, eps_psd=EPS_PSD):
    """The cert_vec of Q's projection in process_noise_state_to_Q_jax (inverse_wishart_jax.py:67)."""
    den = softplus_pos(nu - PROC_BLOCK_DIMS - 1.0)
    Qb = Psi / den[:, None, None] * PROC_BLOCK_MASKS
    Q = np.zeros((D_Z, D_Z))
    for i in range(7):
        s = PROC_BLOCK_STARTS[i]
        e = min(s + 6, D_Z)
        Q[s:e, s:e] = Qb[i][: e - s, : e - s]
    return psd_project(Q, eps_psd)[1]


def iw_meas_mode(nu, Psi, idx):
    """measurement_noise_mean_jax (measurement_noise_iw_jax.py:37-56)."""
    return psd_project(Psi[idx] / (nu[idx] + 3.0 + 1.0))[0]


# ---------------------------------------------------------------------------------------
# a16 HypothesisBarycenterProjection — backend/operators/hypothesis.py:51-236
# ---------------------------------------------------------------------------------------
def hypothesis_barycenter(Ls, hs, zs, weights, floor, eps_psd=EPS_PSD, eps_lift=EPS_LIFT):
    wf = np.maximum(weights, floor)
    adj = float(np.sum(np.abs(wf - weights)))
    wn = wf / np.sum(wf)
    L_raw = np.einsum("k,kij->ij", wn, Ls)
    h = np.einsum("k,ki->i", wn, hs)
    z = np.einsum("k,ki->i", wn, zs)
    L, c = psd_project(L_raw, eps_psd)
    mus = np.stack([chol_solve_lifted(Ls[k], hs[k], eps_lift)[0] for k in range(Ls.shape[0])])
    mom = np.einsum("k,ki->i", wn, mus)
    spread = float(np.sum(wn * np.sum((mus - mom[None]) ** 2, axis=1)))
    K = Ls.shape[0]
    return dict(L=L, h=h, z_lin=z, floor_adjustment=adj, weights=wn, psd_cert=c, spread=spread,
                ess=float(1.0 / np.sum(wn ** 2)), support_frac=float(np.sum(wn > floor) / K),
                mass_eps=adj / K)


# ---------------------------------------------------------------------------------------
# Build-defined legacy bin-path wiring (SURVEY §3.2 "restated"; parity of the wiring itself
# is unpinned — every operator it calls is pinned individually above).
# ---------------------------------------------------------------------------------------
@dataclass
class ScanInput:
    points: np.ndarray
    timestamps: np.ndarray
    weights: np.ndarray
    ring: np.ndarray
    tag: np.ndarray
    imu_stamps: np.ndarray
    imu_gyro: np.ndarray
    imu_accel: np.ndarray
    scan_start: float
    scan_end: float
    t_last: float
    t_scan: float
    dt_sec: float
    odom: "OdomInput" = None


@dataclass
class PipeConfig:
    n_points_cap: int = 65536
    lidar_origin: np.ndarray = field(default_factory=lambda: np.array([-0.065447, -0.100474, 0.108987]))
    tau: float = TAU_SOFT_ASSIGN
    n_bins: int = B_BINS


def scan_hypothesis(b_prev: Belief, scan: ScanInput, Q, io: IOEvidence, mapst: MapStats, mderived,
                    bins, cfg: PipeConfig, Sigma_ga=None):
    """One hypothesis through steps a1-a14 (pipeline.py:316-1591 restated for the bin path).
    io=None: the IMU/odom branch is computed from scan.odom and the IMU window (a9a), with
    Sigma_ga = (Σ_g, Σ_a) the measurement-IW modes (backend_node.py:2021-2023)."""
    o = cfg.lidar_origin
    bud = point_budget_resample(scan.points, scan.timestamps, scan.weights, scan.ring, scan.tag, cfg.n_points_cap)
    pts, ts, ws = bud["points"], bud["timestamps"], bud["weights"]
    bpred, pc = predict_diffusion(b_prev, Q, scan.dt_sec)
    Sig_pred = chol_inverse_lifted(bpred.L)[0]
    sigma_warp = max(math.sqrt(Sig_pred[15, 15]), 0.01)
    w_scan = smooth_window_weights(scan.imu_stamps, scan.scan_start, scan.scan_end, sigma_warp)
    w_int = smooth_window_weights(scan.imu_stamps, scan.t_last, scan.t_scan, sigma_warp)
    mu_inc = chol_solve_lifted(bpred.L, bpred.h)[0]
    bg, ba = mu_inc[9:12], mu_inc[12:15]
    pose0 = world_pose(b_prev)
    rv0 = pose0[3:6]
    pre = preintegrate(scan.imu_stamps, scan.imu_gyro, scan.imu_accel, w_scan, rv0, bg, ba)
    xi = se3_log(pre["delta_pose"])
    dt_imu = imu_dt_mean(scan.imu_stamps)
    wv = w_int * (scan.imu_stamps > 0.0)
    wnv = wv / (np.sum(wv) + EPS_MASS)
    omega_avg = np.einsum("m,mi->i", wnv, scan.imu_gyro - bg[None, :])
    dPsi_meas = np.zeros((3, 3, 3))
    dPsi_meas[0] = iw_meas_gyro_suffstats(scan.imu_gyro, wv, bg, omega_avg, dt_imu)
    dPsi_meas[1] = iw_meas_accel_suffstats(rv0, scan.imu_accel, wv, ba, dt_imu)
    dnu_meas = np.array([1.0, 1.0, 0.0])
    io_parts = None
    if io is None:
        pre_int = preintegrate(scan.imu_stamps, scan.imu_gyro, scan.imu_accel, w_int, rv0, bg, ba)
        dt_int = imu_integration_time(scan.imu_stamps, scan.t_last, scan.t_scan)
        io, io_parts = imu_odom_branch(b_prev, bpred, scan.odom, scan.imu_accel, scan.imu_gyro, w_int, ba, pre_int,
                                       dt_int, dt_imu, omega_avg, scan.dt_sec, Sigma_ga[0], Sigma_ga[1])
    p0, wd, retained = deskew_constant_twist(pts, ts, ws, scan.scan_start, scan.scan_end, xi)
    dirs = point_directions(p0, o)
    sa = bin_soft_assign(dirs, bins, cfg.tau)
    mm = scan_bin_moment_match(p0, None, wd, sa["resp"], None, o)
    R_pred = so3_exp(world_pose(bpred)[3:6])
    t_pred = world_pose(bpred)[0:3]
    mu_dir, kap_m, cen, Sig_c = mderived
    mf = matrix_fisher(R_pred, mm["s_dir"], mm["S_dir_scatter"], mm["N"], mapst.S_dir,
                       mapst.S_dir_scatter, mapst.N_dir)
    tr = planar_translation(t_pred, mm["p_bar"], mm["Sigma_p"], mm["N"], cen, Sig_c, mapst.N_pos,
                            mapst.S_dir_scatter, mapst.N_dir, mf["R_mf"])
    L_lidar = np.zeros((D_Z, D_Z)); h_lidar = np.zeros(D_Z)
    L_lidar[0:3, 0:3] = tr["L_trans"]; h_lidar[0:3] = tr["h_trans"]
    L_lidar[3:6, 3:6] = mf["L_rot"]; h_lidar[3:6] = mf["h_rot"]
    L_raw = io.L + L_lidar
    h_raw = io.h + h_lidar
    # aggregate_certificates([deskew, assign, moments, MF, planar]) then with [odom, imu, gyro]
    ess_ev = (pre["ess"] + sa["ess"] + mm["ess"] + 0.0 + 0.0) / 5.0
    sf_ev = (retained + sa["max_resp"] + mm["support_frac"] + 1.0 + 1.0) / 5.0
    ess_tot = (ess_ev + io.ess.sum()) / 4.0
    sf_tot = (sf_ev + io.support.sum()) / 4.0
    exc_total = max(0.0, io.exc_dt) + max(0.0, io.exc_ex)
    nll = mf["nll_per_ess"] + tr["nll_per_ess"] + io.nll
    beta, dt_asym, z_xy = tempering_beta(L_raw, ess_tot, exc_total)
    L_ev, h_ev = beta * L_raw, beta * h_raw
    Lps, hps, s_dt, s_ex = excitation_scaling(L_ev, bpred.L, bpred.h)
    cond6 = pose6_cond(L_ev)
    alpha = fusion_alpha(cond6, ess_tot, exc_total, dt_asym, z_xy, beta, nll)
    L_post, h_post, fc = info_fusion_additive(Lps, hps, L_ev, h_ev, alpha)
    T = (bud["trig"] + pc["trig"] + io.trig + sa["trig"] + mm["trig"] + mf["trig"] + tr["trig"]
         + trigger(beta=beta) + trigger(dt=1.0 - s_dt, ex=1.0 - s_ex) + trigger(alpha=alpha)
         + trigger(psd=fc[0], alpha=alpha))
    b_post = Belief(bpred.X_anchor.copy(), bpred.z_lin.copy(), L_post, h_post, bpred.stamp_sec)
    b_rec, rc = recompose(b_post, T)
    dPsi_p, dnu_p = iw_process_suffstats(Lps, hps, b_rec.L, b_rec.h)
    z_t = world_pose(b_rec)
    R_t = so3_exp(z_t[3:6])
    t_t = z_t[0:3].copy(); t_t[2] = 0.0
    Sig_pose = chol_inverse_lifted(b_rec.L)[0][0:6, 0:6]
    inc = pose_cov_inflation_pushforward(mm, R_t, t_t, Sig_pose)
    b_fin, dr = anchor_drift(b_rec)
    return dict(belief=b_fin, dPsi_proc=dPsi_p, dnu_proc=dnu_p, dPsi_meas=dPsi_meas, dnu_meas=dnu_meas,
                map_inc=inc, T=T, beta=beta, alpha=alpha, s_dt=s_dt, s_ex=s_ex, xi_body=xi,
                moments=mm, assign=sa, mf=mf, planar=tr, rho=dr["rho"], frob=rc["frobenius_strength"],
                budget=bud, retained=retained, pose=world_pose(b_fin), L_post=L_post, h_post=h_post,
                io=io, io_parts=io_parts, L_ev=L_ev, cond6=cond6, eigmin6=pose6_eigs(L_ev)[0],
                pred_cond=pc["cond"], fusion_cond=np.asarray(fc[2:6]))


@dataclass
class ScanState:
    beliefs: list
    weights: np.ndarray
    nu_proc: np.ndarray
    Psi_proc: np.ndarray
    nu_meas: np.ndarray
    Psi_meas: np.ndarray
    map: MapStats
    scan_count: int = 0


def process_scan(state: ScanState, scan: ScanInput, ios, bins, cfg: PipeConfig, hyp_range=None):
    """backend_node.py:2036-2119 restated for H hypotheses: per-hypothesis pipeline, weighted
    IW accumulation, barycenter combine, one IW apply, hypothesis-0 map update.
    Weight floor = 0.01/H (docs/GC_SLAM.md:122; manifest records it)."""
    H = len(state.beliefs)
    Q = iw_process_Q(state.nu_proc, state.Psi_proc)
    md = map_derived(state.map)
    Sga = (iw_meas_mode(state.nu_meas, state.Psi_meas, 0), iw_meas_mode(state.nu_meas, state.Psi_meas, 1))
    res = [scan_hypothesis(state.beliefs[i], scan, Q, None if ios is None else ios[i], state.map, md, bins, cfg,
                           Sga) for i in range(H)]
    aP = np.zeros((7, 6, 6)); an = np.zeros(7); aM = np.zeros((3, 3, 3)); am = np.zeros(3)
    for i, r in enumerate(res):
        w = float(state.weights[i])
        aP = aP + w * r["dPsi_proc"]; an = an + w * r["dnu_proc"]
        aM = aM + w * r["dPsi_meas"]; am = am + w * r["dnu_meas"]
    new_beliefs = [r["belief"] for r in res]
    comb = hypothesis_barycenter(np.stack([b.L for b in new_beliefs]), np.stack([b.h for b in new_beliefs]),
                                 np.stack([b.z_lin for b in new_beliefs]), state.weights, 0.01 / H)
    wp = float(min(1, state.scan_count))
    nu_p, Psi_p, _ = iw_process_apply(state.nu_proc, state.Psi_proc, wp * aP, wp * an)
    nu_m, Psi_m, _ = iw_meas_apply(state.nu_meas, state.Psi_meas, aM, am)
    new_map = map_forget_and_add(state.map, res[0]["map_inc"])
    st = ScanState(new_beliefs, state.weights.copy(), nu_p, Psi_p, nu_m, Psi_m, new_map, state.scan_count + 1)
    return st, comb, res


# ---------------------------------------------------------------------------------------
# a13 C5 analogue: transform_gaussian_to_world (pipeline.py:1248-1256) + primitive_map_fuse
# (structures/primitive_map.py:992-1163), sequential scatter-add semantics (np.add.at, row order)
# ---------------------------------------------------------------------------------------
def transform_gaussian_to_world(Lb, tb, eb, pose, eps_lift=EPS_LIFT):
    """Rows (K,3,3), (K,3), (K,L,3) -> world frame for z_t = pose = [t, rotvec]."""
    R = so3_exp(pose[3:6])
    t = pose[0:3]
    Lw = np.einsum("ij,kjl,ml->kim", R, Lb, R)
    mu_b = np.linalg.solve(Lb + eps_lift * np.eye(3)[None], tb[..., None])[..., 0]
    mu_w = mu_b @ R.T + t[None]
    tw = np.einsum("kij,kj->ki", Lw, mu_w)
    ew = np.einsum("ij,klj->kli", R, eb)
    return Lw, tw, ew


def primitive_map_fuse(tile: dict, slots, Lambdas, thetas, etas, weights, resp, timestamp, scan_seq, valid=None,
                       colors=None, sources=None, eps_mass=EPS_MASS):
    """Returns a new tile dict (fields as create_empty_tile) after the fuse; out-of-range slots dropped."""
    M = tile["weights"].shape[0]
    slots = np.asarray(slots, np.int64)
    keep = (slots >= 0) & (slots < M)
    r = np.asarray(resp, np.float64) * (1.0 if valid is None else np.asarray(valid, np.float64))
    idx, rk = slots[keep], r[keep]
    out = {k: v.copy() for k, v in tile.items()}
    dL = np.zeros_like(tile["Lambdas"]); np.add.at(dL, idx, rk[:, None, None] * np.asarray(Lambdas)[keep])
    dt = np.zeros_like(tile["thetas"]); np.add.at(dt, idx, rk[:, None] * np.asarray(thetas)[keep])
    de = np.zeros_like(tile["etas"]); np.add.at(de, idx, rk[:, None, None] * np.asarray(etas)[keep])
    w = np.asarray(weights)[keep]
    dw = np.zeros(M); np.add.at(dw, idx, rk * w)
    dr = np.zeros(M); np.add.at(dr, idx, rk)
    out["Lambdas"] = tile["Lambdas"] + dL
    out["thetas"] = tile["thetas"] + dt
    out["etas"] = tile["etas"] + de
    out["weights"] = tile["weights"] + dw
    out["timestamps"][np.unique(idx)] = timestamp
    upd = dr > 0.0
    out["last_supported_scan_seq"] = np.where(upd, scan_seq, tile["last_supported_scan_seq"])
    out["last_update_scan_seq"] = np.where(upd, scan_seq, tile["last_update_scan_seq"])
    if "cam_mass" in tile and sources is not None:
        src = np.asarray(sources)[keep]
        wc = rk * w * (src == 0); wl = rk * w * (src == 1)
        dc = np.zeros(M); np.add.at(dc, idx, wc)
        dl = np.zeros(M); np.add.at(dl, idx, wl)
        out["cam_mass"] = tile["cam_mass"] + dc
        out["lidar_mass"] = tile["lidar_mass"] + dl
        if colors is not None:
            da = np.zeros((M, 3)); np.add.at(da, idx, np.clip(np.asarray(colors)[keep], 0.0, 1.0) * wc[:, None])
            out["rgb_cam_accum"] = tile["rgb_cam_accum"] + da
            dd = np.zeros(M); np.add.at(dd, idx, wc)
            out["rgb_cam_denom"] = tile["rgb_cam_denom"] + dd
    if "cam_mass" in tile:
        est = np.clip(out["rgb_cam_accum"] / np.maximum(out["rgb_cam_denom"][:, None], eps_mass), 0.0, 1.0)
        out["rgb"] = np.where((out["cam_mass"] > 0.0)[:, None], est, 0.5)
        out["colors"] = out["rgb"].copy()
    return out, int(np.unique(idx).shape[0])


def scan_map_slot(mu_w, voxel, M):
    """Spatial hash of the world voxel of each row (uint64 arithmetic, mod M)."""
    v = np.floor(mu_w / voxel).astype(np.int64).view(np.uint64)
    h = (v[:, 0] * np.uint64(73856093)) ^ (v[:, 1] * np.uint64(19349663)) ^ (v[:, 2] * np.uint64(83492791))
    return (h % np.uint64(M)).astype(np.int64)


def scan_map_rows(scan_points, scan_t, scan_w, n_points_cap, t0, t1, h0, nu_meas, Psi_meas, origin, voxel, M,
                  n_lobes=3, eps_mass=EPS_MASS):
    """The C5 in-scan PrimitiveMap update's rows (csrc/gc_scanmap.hip). BUILD-DEFINED, parity
    unpinned: the reference's step 12b (pipeline.py:1236-1327) fuses a measurement batch built
    upstream of the OT association (outside this path) through transform_gaussian_to_world
    (:1248-1256). Here every budgeted point (a1), deskewed with hypothesis 0's twist h0[42:48] (a4),
    is one Gaussian row pushed to the world frame by z_t = h0[0:6] with t_z = 0, its covariance
    Σ_lidar = Ψ_2 / (ν_2 + 4) (measurement_noise_mean_jax's LiDAR block; the IW apply keeps Ψ PSD)
    inflated by J Σ_pose Jᵀ, J = [R | −R[p]×] (a13's inflation, Σ_pose = h0[6:42]); η lobe 0 = R d.
    Returns (slots with -1 for dropped rows, Λ_w, θ_w, η_w, w)."""
    bud = point_budget_resample(scan_points, scan_t, scan_w, None, None, n_points_cap)
    p0, wd, _ = deskew_constant_twist(bud["points"], bud["timestamps"], bud["weights"], t0, t1, h0[42:48])
    valid = (np.arange(n_points_cap) < bud["n_output"]) & (wd > 0.0)
    R = so3_exp(h0[3:6])
    t = np.array([h0[0], h0[1], 0.0])
    mu = np.stack([((R[i, 0] * p0[:, 0] + R[i, 1] * p0[:, 1]) + R[i, 2] * p0[:, 2]) + t[i] for i in range(3)], axis=1)
    # measurement_noise_mean_jax (operators/measurement_noise_iw_jax.py:50-56): PSD-projected mode
    Sl = psd_project(Psi_meas[2] / (nu_meas[2] + 3.0 + 1.0))[0]
    Sp = np.asarray(h0[6:42]).reshape(6, 6)
    K = p0.shape[0]
    J = np.zeros((K, 3, 6))
    J[:, :, 0:3] = R[None]
    J[:, :, 3:6] = -np.einsum("ij,kjl->kil", R, np.stack([skew(p) for p in p0]))
    Sw = (R @ Sl @ R.T)[None] + np.einsum("kia,ab,kjb->kij", J, Sp, J)
    Sw = 0.5 * (Sw + np.swapaxes(Sw, 1, 2))
    Lw = np.linalg.inv(Sw)
    th = np.einsum("kij,kj->ki", Lw, mu)
    eta = np.zeros((K, n_lobes, 3))
    eta[:, 0] = point_directions(p0, np.asarray(origin), eps_mass) @ R.T
    slots = np.where(valid, scan_map_slot(mu, voxel, M), -1)
    return slots, Lw, th, eta, wd


def scan_map_update(tile, rows, timestamp, scan_seq):
    """Fuse the rows of scan_map_rows: responsibility 1, source LiDAR, no colours (primitive_map_fuse
    restated; LiDAR rows leave the colour estimate unchanged)."""
    slots, Lw, th, eta, wd = rows
    K = slots.shape[0]
    return primitive_map_fuse(tile, slots, Lw, th, eta, wd, np.ones(K), timestamp, scan_seq, None, None,
                              np.ones(K, np.int64))


# ---------------------------------------------------------------------------------------
# PrimitiveMap maintenance (structures/primitive_map.py), SURVEY §8f rank 3. A tile is a dict of
# the create_empty_tile fields (valid_mask bool); each function returns a new tile dict.
# ---------------------------------------------------------------------------------------
def empty_tile(m_tile, L=3):
    """create_empty_tile (primitive_map.py:148-175)."""
    return dict(Lambdas=np.zeros((m_tile, 3, 3)), thetas=np.zeros((m_tile, 3)), etas=np.zeros((m_tile, L, 3)),
                weights=np.zeros(m_tile), timestamps=np.zeros(m_tile), created_timestamps=np.zeros(m_tile),
                last_supported_scan_seq=np.zeros(m_tile, np.int64), last_update_scan_seq=np.zeros(m_tile, np.int64),
                primitive_ids=np.zeros(m_tile, np.int64), valid_mask=np.zeros(m_tile, bool),
                colors=np.zeros((m_tile, 3)), cam_mass=np.zeros(m_tile), lidar_mass=np.zeros(m_tile),
                rgb_cam_accum=np.zeros((m_tile, 3)), rgb_cam_denom=np.zeros(m_tile), rgb=np.full((m_tile, 3), 0.5))


def _tile_copy(tile):
    return {k: np.array(v, copy=True) for k, v in tile.items()}


def primitive_map_forget(tile, gamma):
    """primitive_map_forget (primitive_map.py:1314-1390): weights = γ · weights."""
    out = _tile_copy(tile)
    out["weights"] = gamma * tile["weights"]
    return out


def _recency_decay(scan_seq, last_supported, lam):
    dt = np.maximum(np.int64(0), np.int64(scan_seq) - np.asarray(last_supported, np.int64))
    return np.exp(-lam * dt.astype(np.float64))


def primitive_map_recency_inflate(tile, scan_seq, lam, min_scale):
    """primitive_map_recency_inflate (primitive_map.py:1400-1490) for one tile -> (tile, (n_valid,
    Σ(1 - decay), Σ(1/decay - 1)))."""
    valid = np.asarray(tile["valid_mask"], bool)
    decay = np.clip(_recency_decay(scan_seq, tile["last_supported_scan_seq"], lam), float(min_scale), 1.0)
    decay = np.where(valid, decay, 1.0)
    out = _tile_copy(tile)
    out["Lambdas"] = tile["Lambdas"] * decay[:, None, None]
    out["thetas"] = tile["thetas"] * decay[:, None]
    vf = valid.astype(np.float64)
    return out, (float(vf.sum()), float(np.sum((1.0 - decay) * vf)), float(np.sum((1.0 / decay - 1.0) * vf)))


def primitive_map_cull(tile, weight_threshold, max_primitives=None):
    """primitive_map_cull (primitive_map.py:1175-1305) -> (tile, n_culled, mass_dropped)."""
    valid = np.asarray(tile["valid_mask"], bool)
    w = tile["weights"]
    out = _tile_copy(tile)
    count = int(valid.sum())
    if count == 0:
        return out, 0, 0.0
    below = valid & (w < weight_threshold)
    if max_primitives is not None and count - int(below.sum()) > max_primitives:
        sw = np.sort(w * valid.astype(np.float64))[::-1]
        if max_primitives < len(sw):
            below = valid & (w < float(sw[max_primitives]))
    n = int(below.sum())
    if n == 0:
        return out, 0, 0.0
    out["valid_mask"] = valid & ~below
    return out, n, float(np.sum(w * below.astype(np.float64)))


def select_lowest_mass_slots(tile, scan_seq, lam, k):
    """_select_lowest_mass_slots_fixed (primitive_map.py:325-353). jax.lax.sort with the default
    num_keys=1 is a stable sort on the key alone, so ties keep slot order."""
    ret = tile["weights"] * _recency_decay(scan_seq, tile["last_supported_scan_seq"], lam)
    key = np.where(np.asarray(tile["valid_mask"], bool), ret, -np.inf)
    return np.argsort(key, kind="stable")[:k].astype(np.int32)


def primitive_map_insert_masked(tile, Lambdas, thetas, etas, weights, timestamp, valid_new, scan_seq, lam,
                                next_global_id, colors=None, sources=None):
    """primitive_map_insert_masked (primitive_map.py:807-982) -> (tile, n_inserted, new_ids, slots)."""
    w = np.asarray(weights, np.float64).reshape(-1)
    K = w.shape[0]
    slots = select_lowest_mass_slots(tile, scan_seq, lam, K)
    do = np.asarray(valid_new, bool).reshape(-1)
    ids = np.where(do, np.int64(next_global_id) + np.cumsum(do.astype(np.int64)) - 1, np.int64(-1))
    col = np.zeros((K, 3)) if colors is None else np.asarray(colors, np.float64).reshape(K, 3)
    if sources is None:
        is_cam, is_lid = np.zeros(K), np.ones(K)
    else:
        src = np.asarray(sources).reshape(-1)
        is_cam, is_lid = (src == 0).astype(np.float64), (src == 1).astype(np.float64)
    cam, lid = w * is_cam, w * is_lid
    rgb_new = np.where((cam > 0.0)[:, None], np.clip(col, 0.0, 1.0), 0.5)
    out = _tile_copy(tile)
    s = slots[do]
    out["Lambdas"][s] = np.asarray(Lambdas, np.float64).reshape(K, 3, 3)[do]
    out["thetas"][s] = np.asarray(thetas, np.float64).reshape(K, 3)[do]
    out["etas"][s] = np.asarray(etas, np.float64).reshape(K, -1, 3)[do]
    out["weights"][s] = w[do]
    out["timestamps"][s] = float(timestamp)
    out["created_timestamps"][s] = float(timestamp)
    out["last_supported_scan_seq"][s] = scan_seq
    out["last_update_scan_seq"][s] = scan_seq
    out["primitive_ids"][s] = ids[do]
    out["valid_mask"][s] = True
    out["colors"][s] = rgb_new[do]
    out["cam_mass"][s] = cam[do]
    out["lidar_mass"][s] = lid[do]
    out["rgb_cam_accum"][s] = (col * cam[:, None])[do]
    out["rgb_cam_denom"][s] = cam[do]
    out["rgb"][s] = rgb_new[do]
    return out, int(do.sum()), ids, slots


def primitive_map_merge_reduce(tile, merge_threshold, max_pairs, eps_psd=EPS_PSD, eps_lift=EPS_LIFT):
    """primitive_map_merge_reduce (primitive_map.py:1809-2030 -> _merge_reduce_jax :1501-1807)
    -> (tile, n_merged). The caller applies the tile-size budget cap."""
    valid = np.asarray(tile["valid_mask"], bool)
    M = valid.shape[0]
    out = _tile_copy(tile)
    if M < 2 or int(valid.sum()) < 2 or max_pairs <= 0:
        return out, 0
    Lr = tile["Lambdas"] + eps_lift * np.eye(3)[None]
    mu = np.linalg.solve(Lr, tile["thetas"][..., None])[..., 0]
    Sig = np.linalg.inv(Lr)
    det = np.linalg.det(Sig)
    ii, jj = np.triu_indices(M, k=1)
    S = 0.5 * (Sig[ii] + Sig[jj])
    detS = np.linalg.det(S)
    Sinv = np.linalg.inv(S + eps_lift * np.eye(3)[None])
    dmu = (mu[ii] - mu[jj])[:, :, None]
    quad = 0.125 * np.squeeze(np.matmul(np.matmul(dmu.transpose(0, 2, 1), Sinv), dmu), axis=(1, 2))
    with np.errstate(invalid="ignore", divide="ignore"):
        logt = 0.5 * np.log(detS / np.sqrt(det[ii] * det[jj] + 1e-24))
    dist = np.where(valid[ii] & valid[jj], quad + logt, np.inf)
    used = np.zeros(M, bool)
    sel = []
    for idx in np.argsort(dist, kind="stable"):  # select_body (:1560-1585)
        if len(sel) >= max_pairs:
            break
        d, i, j = dist[idx], ii[idx], jj[idx]
        if np.isfinite(d) and d < merge_threshold and not used[i] and not used[j]:
            used[i] = used[j] = True
            sel.append((i, j))
    for i, j in sel:  # merge_body (:1603-1726)
        w1, w2 = out["weights"][i], out["weights"][j]
        ws = w1 + w2
        if not ws > 0.0:
            continue
        mm = (w1 * mu[i] + w2 * mu[j]) / ws
        d1, d2 = (mu[i] - mm)[:, None], (mu[j] - mm)[:, None]
        Sm = (w1 * (Sig[i] + d1 @ d1.T) + w2 * (Sig[j] + d2 @ d2.T)) / ws + eps_psd * np.eye(3)
        Lm = np.linalg.inv(Sm)
        out["Lambdas"][i] = Lm
        out["thetas"][i] = Lm @ mm
        out["etas"][i] = (w1 * out["etas"][i] + w2 * out["etas"][j]) / ws
        cm = out["cam_mass"][i] + out["cam_mass"][j]
        acc = out["rgb_cam_accum"][i] + out["rgb_cam_accum"][j]
        den = out["rgb_cam_denom"][i] + out["rgb_cam_denom"][j]
        rgb = np.clip(acc / max(den, eps_psd), 0.0, 1.0) if cm > 0.0 else np.full(3, 0.5)
        out["cam_mass"][i] = cm
        out["lidar_mass"][i] = out["lidar_mass"][i] + out["lidar_mass"][j]
        out["rgb_cam_accum"][i] = acc
        out["rgb_cam_denom"][i] = den
        out["rgb"][i] = rgb
        out["colors"][i] = rgb
        out["timestamps"][i] = max(out["timestamps"][i], out["timestamps"][j])
        out["created_timestamps"][i] = min(out["created_timestamps"][i], out["created_timestamps"][j])
        out["last_supported_scan_seq"][i] = max(out["last_supported_scan_seq"][i], out["last_supported_scan_seq"][j])
        out["last_update_scan_seq"][i] = max(out["last_update_scan_seq"][i], out["last_update_scan_seq"][j])
        out["weights"][i] = ws
        out["weights"][j] = 0.0
        out["valid_mask"][j] = False
    return out, len(sel)


# ---------------------------------------------------------------------------------------
# Map view + OT association: extract_atlas_map_view
# (structures/primitive_map.py:356-451 + _extract_primitive_map_view_core :475-498) and
# associate_primitives_ot (operators/primitive_association.py:105-553) with the MA-hex tiling
# helpers (common/tiling.py:72-186).
# ---------------------------------------------------------------------------------------
PACK_BITS, PACK_BIAS = 21, 1 << 20
PACK_MASK = (1 << PACK_BITS) - 1


def hex_disk_axial(radius):
    """tiling.py:171-186: axial (q, r) of a hex disk, sorted."""
    r = int(radius)
    out = []
    for q in range(-r, r + 1):
        for rr in range(max(-r, -q - r), min(r, -q + r) + 1):
            out.append((q, rr))
    return sorted(out)


def tile_ids_from_cells(c1, c2, cz):
    """tile_ids_from_cells_jax (tiling.py:148-168): biased, masked 21-bit fields packed in int64."""
    u1 = (np.asarray(c1, np.int64) + PACK_BIAS) & PACK_MASK
    u2 = (np.asarray(c2, np.int64) + PACK_BIAS) & PACK_MASK
    uz = (np.asarray(cz, np.int64) + PACK_BIAS) & PACK_MASK
    return (u1 << (2 * PACK_BITS)) | (u2 << PACK_BITS) | uz


def tile_cells_from_xyz(xyz, h_tile):
    """The cell coordinates of associate_primitives_ot (primitive_association.py:317-323)."""
    h = max(float(h_tile), 1e-12)
    s1 = xyz[:, 0]
    s2 = xyz[:, 0] * 0.5 + xyz[:, 1] * (np.sqrt(3.0) * 0.5)
    return (np.floor(s1 / h).astype(np.int64), np.floor(s2 / h).astype(np.int64),
            np.floor(xyz[:, 2] / h).astype(np.int64))


def extract_atlas_map_view(tiles: dict, tile_ids, m_tile_view, m_tile, L=3, eps_lift=EPS_LIFT, eps_mass=EPS_MASS):
    """tiles: {tile_id: tile dict}; missing ids are empty tiles. Top m_tile_view slots per tile by
    weight (_select_topk_slots_fixed :304-322: a stable sort on -score, invalid = -1e30)."""
    k = int(m_tile_view)
    parts = {n: [] for n in ("slots", "tile", "valid", "Lambdas", "thetas", "etas", "weights", "ids", "last", "rgb")}
    for tid in tile_ids:
        t = tiles.get(int(tid))
        if t is None:
            t = empty_tile(m_tile, L)
        score = np.where(t["valid_mask"], t["weights"], -1e30)
        slots = np.argsort(-score, kind="stable")[:k]
        parts["slots"].append(slots)
        parts["tile"].append(np.full(k, int(tid), np.int64))
        parts["valid"].append(t["valid_mask"][slots])
        parts["Lambdas"].append(t["Lambdas"][slots])
        parts["thetas"].append(t["thetas"][slots])
        parts["etas"].append(t["etas"][slots])
        parts["weights"].append(t["weights"][slots])
        parts["ids"].append(t["primitive_ids"][slots])
        parts["last"].append(t["last_supported_scan_seq"][slots])
        parts["rgb"].append(t["rgb"][slots])
    cat = {n: np.concatenate(v, axis=0) for n, v in parts.items()}
    Lr = cat["Lambdas"] + eps_lift * np.eye(3)[None]
    eta_sum = cat["etas"].sum(axis=1)
    kap = np.linalg.norm(eta_sum, axis=1)
    return dict(candidate_tile_ids=cat["tile"], candidate_slots=cat["slots"].astype(np.int64),
                valid_mask=cat["valid"].astype(bool), tile_ids=np.asarray(tile_ids, np.int64), m_tile_view=k,
                positions=np.linalg.solve(Lr, cat["thetas"][..., None])[..., 0], covariances=np.linalg.inv(Lr),
                directions=eta_sum / (kap[:, None] + eps_mass), kappas=kap, weights=cat["weights"],
                primitive_ids=cat["ids"], last_supported_scan_seq=cat["last"], etas=cat["etas"], colors=cat["rgb"])


def _A_vmf(k, eps=1e-12):
    """_A_vmf_vec_jax (primitive_association.py:141-149)."""
    k = np.maximum(np.asarray(k, np.float64), eps)
    with np.errstate(over="ignore", invalid="ignore"):
        log_sinh = np.where(k > 20.0, k - np.log(2.0),
                            np.where(k >= 1e-2, np.log(np.sinh(np.minimum(k, 20.0))), np.log(k + k ** 3 / 6.0)))
    return np.log(4.0 * np.pi) + log_sinh - np.log(k)


def ot_cost(mp, md, mk, vp, vd, vk, beta=0.5, eig_min=1e-12):
    """_compute_sparse_cost_matrix_jax (:152-197) on gathered candidates: mp (N,3), vp (N,C,3)."""
    diff = mp[:, None, :] - vp
    d_pos = np.sum(diff * diff, axis=-1)
    km = 0.5 * np.linalg.norm(mk[:, None, None] * md[:, None, :] + vk[:, :, None] * vd, axis=-1)
    bc = np.exp(_A_vmf(np.maximum(km, eig_min), eig_min) -
                0.5 * (_A_vmf(np.maximum(mk[:, None], eig_min), eig_min) + _A_vmf(np.maximum(vk, eig_min), eig_min)))
    d_dir = np.maximum(0.0, 1.0 - bc)
    d_dir = np.where((mk[:, None] > 0.0) & (vk > 0.0), d_dir, 0.0)
    return d_pos + float(beta) * d_dir


OT_DEFAULTS = dict(k_assoc=8, k_sinkhorn=50, beta=0.5, epsilon=0.1, tau_a=0.5, tau_b=0.5, cost_subtract_row_min=True,
                   weight_proportional=False, eps_mass=EPS_MASS, h_tile=2.0, r_xy=1, r_z=0, scan_seq=0,
                   recency_decay_lambda=0.02)


def associate_primitives_ot(meas: dict, view: dict, cfg: dict = None, eps_lift=EPS_LIFT, eps_mass=EPS_MASS):
    """associate_primitives_ot (primitive_association.py:239-553): meas = {Lambdas, thetas, etas,
    weights, valid_mask}. Returns the result arrays and the OT cert scalars."""
    c = dict(OT_DEFAULTS, **(cfg or {}))
    K = int(c["k_assoc"])
    valid = np.asarray(meas["valid_mask"], bool)
    N = valid.shape[0]
    zeros = dict(responsibilities=np.zeros((N, K)), candidate_pool_indices=np.zeros((N, K), np.int32),
                 candidate_tile_ids=np.zeros((N, K), np.int64), candidate_slots=np.zeros((N, K), np.int64),
                 row_masses=np.zeros(N), cost_matrix=np.zeros((N, K)))
    if valid.sum() == 0 or view["valid_mask"].sum() == 0:
        return zeros, None
    Lr = meas["Lambdas"] + eps_lift * np.eye(3)[None]
    mp = np.linalg.solve(Lr, meas["thetas"][..., None])[..., 0]
    es = meas["etas"].sum(axis=1)
    mk = np.linalg.norm(es, axis=1)
    md = es / (np.linalg.norm(es, axis=1, keepdims=True) + eps_mass)
    vf = valid.astype(np.float64)
    disk = hex_disk_axial(c["r_xy"])
    dq = np.array([d[0] for d in disk], np.int64)
    dr = np.array([d[1] for d in disk], np.int64)
    dz = np.arange(-int(c["r_z"]), int(c["r_z"]) + 1, dtype=np.int64)
    c1, c2, cz = tile_cells_from_xyz(mp, c["h_tile"])
    g1 = c1[:, None, None] + dq[None, None, :] + 0 * dz[None, :, None]
    g2 = c2[:, None, None] + dr[None, None, :] + 0 * dz[None, :, None]
    gz = cz[:, None, None] + dz[None, :, None] + 0 * dq[None, None, :]
    st = tile_ids_from_cells(g1, g2, gz).reshape(N, -1)
    pool_tiles = view["tile_ids"]
    kv = int(view["m_tile_view"])
    eq = st[:, :, None] == pool_tiles[None, None, :]
    has = eq.any(axis=2)
    tix = np.where(has, eq.argmax(axis=2), 0)
    pool = ((tix * kv)[:, :, None] + np.arange(kv)[None, None, :]).reshape(N, -1)
    cost_pool = ot_cost(mp, md, mk, view["positions"][pool], view["directions"][pool], view["kappas"][pool], c["beta"])
    pv = view["valid_mask"][pool] & np.repeat(has, kv, axis=1)
    cost_pool = np.where(pv, cost_pool, 1e12)
    order = np.argsort(cost_pool, axis=1, kind="stable")  # lax.sort, num_keys=1: cost only, stable
    cand = np.take_along_axis(pool, order, axis=1)[:, :K].astype(np.int32)
    cand = np.where(valid[:, None], cand, 0).astype(np.int32)
    C = ot_cost(mp, md, mk, view["positions"][cand], view["directions"][cand], view["kappas"][cand], c["beta"])
    dt = np.maximum(0, np.int64(c["scan_seq"]) - view["last_supported_scan_seq"][cand]).astype(np.float64)
    C = C + float(c["epsilon"]) * float(c["recency_decay_lambda"]) * dt
    if c["cost_subtract_row_min"]:
        C = C - C.min(axis=1, keepdims=True)
    if c["weight_proportional"]:
        wv = vf * np.asarray(meas["weights"], np.float64)
        sum_a = max(wv.sum(), c["eps_mass"])
        a = wv / sum_a
    else:
        sum_a = max(vf.sum(), c["eps_mass"])
        a = vf / sum_a
    b = np.ones(K) / K
    eps = max(float(c["epsilon"]), 1e-12)
    Km = np.exp(-C / eps)
    ua, vb = 1.0 / (1.0 + c["tau_a"] / eps), 1.0 / (1.0 + c["tau_b"] / eps)
    u, v = np.ones(N), np.ones(K)
    for _ in range(int(c["k_sinkhorn"])):
        u = (a / (Km @ v + 1e-12)) ** ua
        v = (b / (Km.T @ u + 1e-12)) ** vb
    pi = u[:, None] * Km * v[None, :]
    rows = pi.sum(axis=1)
    res = dict(responsibilities=pi * valid[:, None], candidate_pool_indices=cand,
               candidate_tile_ids=view["candidate_tile_ids"][cand], candidate_slots=view["candidate_slots"][cand],
               row_masses=rows, cost_matrix=C)
    em = c["eps_mass"]
    cols = pi.sum(axis=0)
    cert = dict(marginal_defect_a=float(np.linalg.norm(rows - a)), marginal_defect_b=float(np.linalg.norm(cols - b)),
                transport_mass_total=float(pi.sum()), sum_a=float(sum_a), sum_b=float(b.sum()),
                sum_m=float(rows.sum()), sum_novel=float(np.maximum(a - rows, 0.0).sum()),
                ess=float(rows.sum() ** 2 / (np.sum(rows ** 2) + em)), nonzero_a=int(np.sum(a > em)),
                nonzero_b=int(np.sum(b > em)), total_cost=float(np.sum(pi * C)))
    return res, cert
