"""IMU/odom evidence factors of the GC-SLAM v2 pipeline (pipeline.py:595-776) on the GPU.

Reference-named drop-ins, each returning ``(Result, CertBundle, ExpectedEffect)`` like the
reference operator it replaces:

- ``odom_quadratic_evidence``  backend/operators/odom_evidence.py:87-154
- ``imu_vmf_gravity_evidence_time_resolved``  imu_evidence.py:402-559
- ``imu_dependence_inflation``  imu_evidence.py:562-589
- ``imu_gyro_rotation_evidence``  imu_gyro_evidence.py:103-163
- ``imu_preintegration_factor``  imu_preintegration_factor.py:46-180
- ``planar_z_prior`` / ``velocity_z_prior``  planar_prior.py:55-195
- ``odom_velocity_evidence`` / ``odom_yawrate_evidence``  odom_twist_evidence.py:58-225
- ``pose_twist_kinematic_consistency`` / ``odom_dependence_inflation``  odom_twist_evidence.py:251-430

Every arithmetic step runs in libgcslam (``gc_io_factor_batch`` — one thread per item — and
``gc_imu_vmf_gravity_tr_batch``, one workgroup per item); the batched pipeline runs the same
device code for all hypotheses in one launch. ``io_factor_batch`` is the H-item entry.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import numpy as np

from .. import _abi
from ..certificates import (CertBundle, ConditioningCert, ExpectedEffect, InfluenceCert, MismatchCert,
                            SupportCert)
from ..constants import (D_Z, GC_CHART_ID, GC_EPS_LIFT, GC_EPS_MASS, GC_EPS_PSD, GC_PLANAR_VZ_SIGMA)

_N2 = D_Z * D_Z


def io_factor_batch(kind: int, rows: np.ndarray, ctx=None) -> np.ndarray:
    """rows (H, k <= GC_IOF_IN) in the kind's input layout (include/gcslam.h GC_IOF_*) ->
    (H, GC_IOF_OUT) = L (22,22) | h (22) | extras (16)."""
    ctx = ctx or _abi.default_context()
    rows = np.atleast_2d(np.asarray(rows, dtype=np.float64))
    H, k = rows.shape
    if k > _abi.GC_IOF_IN:
        raise ValueError(f"factor row has {k} > {_abi.GC_IOF_IN} entries")
    buf = np.zeros((H, _abi.GC_IOF_IN))
    buf[:, :k] = rows
    din = _abi.DeviceArray.from_host(ctx, buf)
    dout = _abi.DeviceArray(ctx, (H, _abi.GC_IOF_OUT))
    _abi.call("gc_io_factor_batch", ctx.handle, int(kind), H, din.ptr, dout.ptr, ctx=ctx)
    return dout.download()


def _split(out_row):
    return out_row[:_N2].reshape(D_Z, D_Z).copy(), out_row[_N2:_N2 + D_Z].copy(), out_row[_N2 + D_Z:]


def _v(a, n):
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    if a.shape[0] != n:
        raise ValueError(f"expected {n} values, got {a.shape[0]}")
    return a


def _m(a, n):
    a = np.asarray(a, dtype=np.float64)
    if a.size != n * n:
        raise ValueError(f"expected a ({n},{n}) matrix, got shape {a.shape}")
    return a.reshape(-1)


def _cond(e_min, e_max, nnc, cond=None):
    return ConditioningCert(eig_min=float(e_min), eig_max=float(e_max),
                            cond=float(e_max / max(e_min, 1e-18) if cond is None else cond),
                            near_null_count=int(nnc))


# ------------------------------------------------------------------------------ odometry pose
@dataclass
class OdomEvidenceResult:
    L_odom: np.ndarray
    h_odom: np.ndarray
    delta_z_star: np.ndarray


def odom_quadratic_evidence(belief_pred_pose, odom_pose, odom_cov_se3, eps_psd: float = GC_EPS_PSD,
                            eps_lift: float = GC_EPS_LIFT, chart_id: str = GC_CHART_ID, anchor_id: str = "",
                            ctx=None) -> Tuple[OdomEvidenceResult, CertBundle, ExpectedEffect]:
    row = np.concatenate([_v(belief_pred_pose, 6), _v(odom_pose, 6), _m(odom_cov_se3, 6), [eps_psd, eps_lift]])
    L, h, ex = _split(io_factor_batch(_abi.GC_IOF_ODOM_QUADRATIC, row, ctx)[0])
    dz = np.zeros(D_Z)
    dz[0:6] = ex[0:6]
    nll = float(ex[6])
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=["OdomEvidenceGaussian"],
                                    conditioning=_cond(ex[8], ex[9], ex[11], ex[10]),
                                    mismatch=MismatchCert(nll_per_ess=nll, directional_score=0.0),
                                    influence=InfluenceCert.identity().with_overrides(lift_strength=float(ex[7])))
    return (OdomEvidenceResult(L_odom=L, h_odom=h, delta_z_star=dz), cert,
            ExpectedEffect(objective_name="odom_quadratic_nll_proxy", predicted=nll, realized=None))


# ------------------------------------------------------------------------------ IMU gravity
@dataclass
class TimeResolvedImuResult:
    L_imu: np.ndarray
    h_imu: np.ndarray
    kappa: float
    ess_weighted: float
    ess_raw: float
    mean_reliability: float
    transport_sigma: float


@dataclass
class ImuDependenceInflationResult:
    scale: float


def imu_vmf_gravity_evidence_time_resolved_batch(rotvec, imu_accel, imu_gyro, weights, accel_bias, gravity_W,
                                                 dt_imu, eps_psd=GC_EPS_PSD, eps_mass=GC_EPS_MASS, ctx=None):
    """H items over one IMU window: rotvec (H,3), accel/gyro (M,3), weights (H,M), bias (H,3)
    -> (H, GC_IOF_OUT) rows (extras layout: include/gcslam.h gc_imu_vmf_gravity_tr_batch)."""
    ctx = ctx or _abi.default_context()
    rv = np.atleast_2d(np.asarray(rotvec, np.float64))
    H = rv.shape[0]
    acc = np.ascontiguousarray(imu_accel, np.float64)
    M = acc.shape[0]
    w = np.ascontiguousarray(np.broadcast_to(np.asarray(weights, np.float64), (H, M)))
    ba = np.ascontiguousarray(np.broadcast_to(np.asarray(accel_bias, np.float64), (H, 3)))
    d = _abi.upload_many(ctx, (rv, acc, np.ascontiguousarray(imu_gyro, np.float64), w, ba))
    out = _abi.DeviceArray(ctx, (H, _abi.GC_IOF_OUT))
    g, gp = _abi.f64p(_v(gravity_W, 3))
    _abi.call("gc_imu_vmf_gravity_tr_batch", ctx.handle, H, M, *[x.ptr for x in d], gp, float(dt_imu),
              float(eps_psd), float(eps_mass), out.ptr, ctx=ctx)
    return out.download()


def imu_vmf_gravity_evidence_time_resolved(rotvec_world_body, imu_accel, imu_gyro, weights, accel_bias, gravity_W,
                                           dt_imu: float, eps_psd: float, eps_mass: float, chart_id: str,
                                           anchor_id: str, ctx=None
                                           ) -> Tuple[TimeResolvedImuResult, CertBundle, ExpectedEffect]:
    acc = np.asarray(imu_accel, np.float64)
    if acc.ndim != 2 or acc.shape[1] != 3 or np.asarray(imu_gyro).shape != acc.shape:
        raise ValueError(f"imu_accel/imu_gyro must be (M,3), got {acc.shape} / {np.asarray(imu_gyro).shape}")
    L, h, ex = _split(imu_vmf_gravity_evidence_time_resolved_batch(
        _v(rotvec_world_body, 3)[None], acc, imu_gyro, _v(weights, acc.shape[0])[None], _v(accel_bias, 3)[None],
        gravity_W, dt_imu, eps_psd, eps_mass, ctx)[0])
    kappa, ess_w, ess_raw, mrel, sigma, Rbar, nll, nll_pe, psd_d = (float(x) for x in ex[0:9])
    cert = CertBundle.create_approx(
        chart_id=chart_id, anchor_id=anchor_id,
        triggers=["ImuAccelDirectionTimeResolved", "TransportConsistencyWeighting", "KappaLowRApproximation"],
        conditioning=_cond(ex[9], ex[10], ex[12], ex[11]),
        support=SupportCert(ess_total=ess_w, support_frac=mrel),
        mismatch=MismatchCert(nll_per_ess=nll_pe, directional_score=Rbar),
        influence=InfluenceCert.identity().with_overrides(psd_projection_delta=psd_d,
                                                          mass_epsilon_ratio=ess_w / (ess_raw + eps_mass),
                                                          trust_alpha=mrel))
    res = TimeResolvedImuResult(L_imu=L, h_imu=h, kappa=kappa, ess_weighted=ess_w, ess_raw=ess_raw,
                                mean_reliability=mrel, transport_sigma=sigma)
    return res, cert, ExpectedEffect(objective_name="imu_accel_direction_time_resolved_nll_proxy", predicted=nll,
                                     realized=None)


def _dependence(kind, row, trig, objective, chart_id, anchor_id, ctx):
    scale = float(io_factor_batch(kind, row, ctx)[0, _N2 + D_Z])
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=[trig],
                                    influence=InfluenceCert.identity().with_overrides(trust_alpha=scale))
    return scale, cert, ExpectedEffect(objective_name=objective, predicted=scale, realized=scale)


def imu_dependence_inflation(transport_sigma: float, eps_mass: float, chart_id: str, anchor_id: str, ctx=None
                             ) -> Tuple[ImuDependenceInflationResult, CertBundle, ExpectedEffect]:
    s, cert, eff = _dependence(_abi.GC_IOF_IMU_DEPENDENCE, [float(transport_sigma), float(eps_mass)],
                               "ImuDependenceInflation", "imu_dependence_inflation", chart_id, anchor_id, ctx)
    return ImuDependenceInflationResult(scale=s), cert, eff


# ------------------------------------------------------------------------------ IMU gyro / preint
@dataclass
class ImuGyroEvidenceResult:
    L_gyro: np.ndarray
    h_gyro: np.ndarray
    r_rot: np.ndarray


def imu_gyro_rotation_evidence(rotvec_start_WB, rotvec_end_pred_WB, delta_rotvec_meas, Sigma_g, dt_int: float,
                               eps_psd: float = GC_EPS_PSD, eps_lift: float = GC_EPS_LIFT,
                               chart_id: str = GC_CHART_ID, anchor_id: str = "initial", ctx=None
                               ) -> Tuple[ImuGyroEvidenceResult, CertBundle, ExpectedEffect]:
    row = np.concatenate([_v(rotvec_start_WB, 3), _v(rotvec_end_pred_WB, 3), _v(delta_rotvec_meas, 3),
                          _m(Sigma_g, 3), [dt_int, eps_psd, eps_lift, GC_EPS_MASS]])
    L, h, ex = _split(io_factor_batch(_abi.GC_IOF_IMU_GYRO_ROTATION, row, ctx)[0])
    nll = float(ex[3])
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=["ImuGyroRotationGaussian"],
                                    conditioning=_cond(ex[5], ex[6], ex[7]),
                                    mismatch=MismatchCert(nll_per_ess=nll, directional_score=0.0),
                                    influence=InfluenceCert.identity().with_overrides(lift_strength=float(ex[4])))
    return (ImuGyroEvidenceResult(L_gyro=L, h_gyro=h, r_rot=ex[0:3].copy()), cert,
            ExpectedEffect(objective_name="imu_gyro_rotation_nll_proxy", predicted=nll, realized=None))


@dataclass
class ImuPreintegrationFactorResult:
    L_imu_preint: np.ndarray
    h_imu_preint: np.ndarray
    r_vel: np.ndarray
    r_pos: np.ndarray


def imu_preintegration_factor(p_start_world, rotvec_start_WB, v_start_world, p_end_pred_world, v_end_pred_world,
                              delta_v_body, delta_p_body, Sigma_a, dt_int: float, eps_psd: float = GC_EPS_PSD,
                              eps_lift: float = GC_EPS_LIFT, chart_id: str = GC_CHART_ID, anchor_id: str = "initial",
                              ctx=None) -> Tuple[ImuPreintegrationFactorResult, CertBundle, ExpectedEffect]:
    row = np.concatenate([_v(p_start_world, 3), _v(rotvec_start_WB, 3), _v(v_start_world, 3),
                          _v(p_end_pred_world, 3), _v(v_end_pred_world, 3), _v(delta_v_body, 3),
                          _v(delta_p_body, 3), _m(Sigma_a, 3), [dt_int, eps_psd, eps_lift, GC_EPS_MASS]])
    L, h, ex = _split(io_factor_batch(_abi.GC_IOF_IMU_PREINT_FACTOR, row, ctx)[0])
    nll = float(ex[6])
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=["ImuPreintegrationVelPos"],
                                    conditioning=_cond(ex[8], ex[9], ex[11], ex[10]),
                                    mismatch=MismatchCert(nll_per_ess=nll, directional_score=0.0),
                                    influence=InfluenceCert.identity().with_overrides(lift_strength=float(ex[7])))
    return (ImuPreintegrationFactorResult(L_imu_preint=L, h_imu_preint=h, r_vel=ex[0:3].copy(), r_pos=ex[3:6].copy()),
            cert, ExpectedEffect(objective_name="imu_preint_nll_proxy", predicted=nll, realized=None))


# ------------------------------------------------------------------------------ planar priors
@dataclass
class PlanarPriorResult:
    L_planar: np.ndarray
    h_planar: np.ndarray
    r_z: float


@dataclass
class VelocityZPriorResult:
    L_vz: np.ndarray
    h_vz: np.ndarray
    v_z: float


def planar_z_prior(belief_pred_pose, z_ref: float, sigma_z: float, eps_psd: float = GC_EPS_PSD,
                   chart_id: str = GC_CHART_ID, anchor_id: str = "", ctx=None
                   ) -> Tuple[PlanarPriorResult, CertBundle, ExpectedEffect]:
    row = np.concatenate([_v(belief_pred_pose, 6), [z_ref, sigma_z]])
    L, h, ex = _split(io_factor_batch(_abi.GC_IOF_PLANAR_Z_PRIOR, row, ctx)[0])
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=["PlanarZPrior"],
                                    influence=InfluenceCert.identity())
    return (PlanarPriorResult(L_planar=L, h_planar=h, r_z=float(ex[0])), cert,
            ExpectedEffect(objective_name="planar_z_prior_nll", predicted=float(ex[1]), realized=None))


def velocity_z_prior(v_z_pred: float, sigma_vz: float = GC_PLANAR_VZ_SIGMA, chart_id: str = GC_CHART_ID,
                     anchor_id: str = "", ctx=None) -> Tuple[VelocityZPriorResult, CertBundle, ExpectedEffect]:
    L, h, ex = _split(io_factor_batch(_abi.GC_IOF_VELOCITY_Z_PRIOR, [float(v_z_pred), float(sigma_vz)], ctx)[0])
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=["VelocityZPrior"],
                                    influence=InfluenceCert.identity())
    return (VelocityZPriorResult(L_vz=L, h_vz=h, v_z=float(ex[0])), cert,
            ExpectedEffect(objective_name="velocity_z_prior_nll", predicted=float(ex[1]), realized=None))


# ------------------------------------------------------------------------------ odometry twist
@dataclass
class OdomVelocityEvidenceResult:
    L_vel: np.ndarray
    h_vel: np.ndarray
    r_vel: np.ndarray


@dataclass
class OdomYawRateEvidenceResult:
    L_wz: np.ndarray
    h_wz: np.ndarray
    r_wz: float


@dataclass
class PoseTwistConsistencyResult:
    L_consistency: np.ndarray
    h_consistency: np.ndarray
    r_trans: np.ndarray
    r_rot: np.ndarray


@dataclass
class OdomDependenceInflationResult:
    scale: float


def odom_velocity_evidence(v_pred_world, R_world_body, v_odom_body, Sigma_v, eps_psd: float = GC_EPS_PSD,
                           eps_lift: float = GC_EPS_LIFT, chart_id: str = GC_CHART_ID, anchor_id: str = "",
                           ctx=None) -> Tuple[OdomVelocityEvidenceResult, CertBundle, ExpectedEffect]:
    row = np.concatenate([_v(v_pred_world, 3), _m(R_world_body, 3), _v(v_odom_body, 3), _m(Sigma_v, 3),
                          [eps_psd, eps_lift]])
    L, h, ex = _split(io_factor_batch(_abi.GC_IOF_ODOM_VELOCITY, row, ctx)[0])
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=["OdomVelocityEvidence"],
                                    conditioning=_cond(ex[5], ex[6], ex[8], ex[7]),
                                    influence=InfluenceCert.identity().with_overrides(lift_strength=float(ex[4])))
    return (OdomVelocityEvidenceResult(L_vel=L, h_vel=h, r_vel=ex[0:3].copy()), cert,
            ExpectedEffect(objective_name="odom_velocity_nll", predicted=float(ex[3]), realized=None))


def odom_yawrate_evidence(omega_z_pred: float, omega_z_odom: float, sigma_wz: float, chart_id: str = GC_CHART_ID,
                          anchor_id: str = "", ctx=None) -> Tuple[OdomYawRateEvidenceResult, CertBundle, ExpectedEffect]:
    row = [float(omega_z_pred), float(omega_z_odom), float(sigma_wz)]
    L, h, ex = _split(io_factor_batch(_abi.GC_IOF_ODOM_YAWRATE, row, ctx)[0])
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=["OdomYawRateEvidence"],
                                    influence=InfluenceCert.identity())
    return (OdomYawRateEvidenceResult(L_wz=L, h_wz=h, r_wz=float(ex[0])), cert,
            ExpectedEffect(objective_name="odom_yawrate_nll", predicted=float(ex[1]), realized=None))


def pose_twist_kinematic_consistency(pose_prev, pose_curr, v_body, omega_body, dt: float, Sigma_v, Sigma_omega,
                                     eps_psd: float = GC_EPS_PSD, eps_lift: float = GC_EPS_LIFT,
                                     chart_id: str = GC_CHART_ID, anchor_id: str = "", ctx=None
                                     ) -> Tuple[PoseTwistConsistencyResult, CertBundle, ExpectedEffect]:
    row = np.concatenate([_v(pose_prev, 6), _v(pose_curr, 6), _v(v_body, 3), _v(omega_body, 3), [float(dt)],
                          _m(Sigma_v, 3), _m(Sigma_omega, 3), [eps_psd, eps_lift]])
    L, h, ex = _split(io_factor_batch(_abi.GC_IOF_KINEMATIC, row, ctx)[0])
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id,
                                    triggers=["PoseTwistKinematicConsistency"],
                                    conditioning=_cond(ex[8], ex[9], 0, ex[10]),
                                    influence=InfluenceCert.identity().with_overrides(lift_strength=float(ex[7])))
    return (PoseTwistConsistencyResult(L_consistency=L, h_consistency=h, r_trans=ex[0:3].copy(),
                                       r_rot=ex[3:6].copy()), cert,
            ExpectedEffect(objective_name="pose_twist_consistency_nll", predicted=float(ex[6]), realized=None))


def odom_dependence_inflation(r_trans, r_rot, eps_mass: float, chart_id: str, anchor_id: str, ctx=None
                              ) -> Tuple[OdomDependenceInflationResult, CertBundle, ExpectedEffect]:
    row = np.concatenate([_v(r_trans, 3), _v(r_rot, 3), [float(eps_mass)]])
    s, cert, eff = _dependence(_abi.GC_IOF_ODOM_DEPENDENCE, row, "OdomDependenceInflation",
                               "odom_dependence_inflation", chart_id, anchor_id, ctx)
    return OdomDependenceInflationResult(scale=s), cert, eff
