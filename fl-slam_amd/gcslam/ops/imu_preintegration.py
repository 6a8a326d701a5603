"""IMU soft windows and weighted preintegration (backend/operators/imu_preintegration.py:19-147)
and the IMU measurement-noise IW statistics (measurement_noise_iw_jax.py:131-218) on the GPU."""

from __future__ import annotations

import numpy as np

from .. import _abi
from ..constants import GC_EPS_MASS, GC_EPS_PSD, GC_GRAVITY_W, GC_MAX_IMU_PREINT_LEN


def smooth_window_weights(imu_stamps, scan_start_time: float, scan_end_time: float, sigma: float, ctx=None):
    """w_i = σ((t_i − t0)/s)·σ((t1 − t_i)/s)·(1 − 1e-12) + 1e-12, s = max(σ, 1e-6)."""
    ctx = ctx or _abi.default_context()
    t = np.ascontiguousarray(imu_stamps, dtype=np.float64).reshape(-1)
    M = t.shape[0]
    dt_, dw = _abi.DeviceArray.from_host(ctx, t), _abi.DeviceArray(ctx, M)
    _abi.call("gc_smooth_window_weights", ctx.handle, M, dt_.ptr, float(scan_start_time), float(scan_end_time),
              float(sigma), dw.ptr, ctx=ctx)
    return dw.download()


def preintegrate_imu_batch(imu_stamps, imu_gyro, imu_accel, weights, rotvec_start_WB, gyro_bias, accel_bias,
                           gravity_W=GC_GRAVITY_W, ctx=None):
    """Shared IMU window, H (weights, start rotation, biases) -> (H, 32) rows (include/gcslam.h
    GC_PREINT_OUT). weights may be (M,) (shared) or (H, M)."""
    ctx = ctx or _abi.default_context()
    t = np.ascontiguousarray(imu_stamps, dtype=np.float64).reshape(-1)
    M = t.shape[0]
    if not 1 <= M <= GC_MAX_IMU_PREINT_LEN:
        raise ValueError(f"IMU window must hold 1..{GC_MAX_IMU_PREINT_LEN} samples, got {M}")
    g = np.ascontiguousarray(imu_gyro, dtype=np.float64).reshape(M, 3)
    a = np.ascontiguousarray(imu_accel, dtype=np.float64).reshape(M, 3)
    r0 = np.ascontiguousarray(rotvec_start_WB, dtype=np.float64).reshape(-1, 3)
    H = r0.shape[0]
    bg = np.ascontiguousarray(np.broadcast_to(np.asarray(gyro_bias, np.float64).reshape(-1, 3), (H, 3)))
    ba = np.ascontiguousarray(np.broadcast_to(np.asarray(accel_bias, np.float64).reshape(-1, 3), (H, 3)))
    w = np.ascontiguousarray(weights, dtype=np.float64)
    stride = 0 if w.ndim == 1 else M
    if w.reshape(-1).shape[0] not in (M, H * M):
        raise ValueError("weights must be (M,) or (H, M)")
    dev = _abi.upload_many(ctx, (t, g, a, w, r0, bg, ba))
    out = _abi.DeviceArray(ctx, (H, _abi.GC_PREINT_OUT))
    ga, gp = _abi.f64p(gravity_W)
    _abi.call("gc_preintegrate_imu_batch", ctx.handle, H, M, dev[0].ptr, dev[1].ptr, dev[2].ptr, dev[3].ptr, stride,
              dev[4].ptr, dev[5].ptr, dev[6].ptr, gp, out.ptr, ctx=ctx)
    return out.download()


def preintegrate_imu_relative_pose_jax(imu_stamps, imu_gyro, imu_accel, weights, rotvec_start_WB, gyro_bias,
                                       accel_bias, gravity_W, ctx=None):
    """Same 9-tuple as the reference: (delta_pose, delta_R, delta_p, delta_v, ess, a_body_mean,
    a_world_nog_mean, a_world_mean, dt_eff_sum)."""
    o = preintegrate_imu_batch(imu_stamps, imu_gyro, imu_accel, weights, np.asarray(rotvec_start_WB)[None],
                               gyro_bias, accel_bias, gravity_W, ctx)[0]
    return (o[0:6], o[6:15].reshape(3, 3), o[15:18], o[18:21], float(o[21]), o[22:25], o[25:28], o[28:31],
            float(o[31]))


def imu_meas_iw_suffstats_batch(imu_gyro, imu_accel, weights, gyro_bias, accel_bias, omega_avg, rotvec_start_WB,
                                dt_imu: float, eps_mass=GC_EPS_MASS, eps_psd=GC_EPS_PSD, ctx=None):
    """(H, 2, 3, 3): [gyro dΨ, accel dΨ] per hypothesis (shared IMU window)."""
    ctx = ctx or _abi.default_context()
    g = np.ascontiguousarray(imu_gyro, dtype=np.float64).reshape(-1, 3)
    M = g.shape[0]
    a = np.ascontiguousarray(imu_accel, dtype=np.float64).reshape(M, 3)
    w = np.ascontiguousarray(weights, dtype=np.float64).reshape(M)
    rows = [np.ascontiguousarray(np.asarray(x, np.float64).reshape(-1, 3)) for x in
            (gyro_bias, accel_bias, omega_avg, rotvec_start_WB)]
    H = max(r.shape[0] for r in rows)
    rows = [np.ascontiguousarray(np.broadcast_to(r, (H, 3))) for r in rows]
    dev = _abi.upload_many(ctx, [g, a, w] + rows)
    out = _abi.DeviceArray(ctx, (H, 18))
    _abi.call("gc_imu_meas_iw_suffstats_batch", ctx.handle, H, M, *[d.ptr for d in dev], float(dt_imu),
              float(eps_mass), float(eps_psd), out.ptr, ctx=ctx)
    return out.download().reshape(H, 2, 3, 3)


def imu_gyro_meas_iw_suffstats_from_avg_rate_jax(imu_gyro, weights, gyro_bias, omega_avg, dt_imu, ctx=None):
    """measurement_noise_iw_jax.py:131-171 -> dΨ_gyro (3,3)."""
    z3 = np.zeros(3)
    g = np.asarray(imu_gyro, np.float64)
    return imu_meas_iw_suffstats_batch(g, np.zeros_like(g), weights, gyro_bias, z3, omega_avg, z3, dt_imu,
                                       ctx=ctx)[0, 0]


def imu_accel_meas_iw_suffstats_from_gravity_dir_jax(rotvec_start_WB, imu_accel, weights, accel_bias, dt_imu,
                                                     ctx=None):
    """measurement_noise_iw_jax.py:174-218 -> dΨ_accel (3,3)."""
    z3 = np.zeros(3)
    a = np.asarray(imu_accel, np.float64)
    return imu_meas_iw_suffstats_batch(np.zeros_like(a), a, weights, z3, accel_bias, z3, rotvec_start_WB, dt_imu,
                                       ctx=ctx)[0, 1]
