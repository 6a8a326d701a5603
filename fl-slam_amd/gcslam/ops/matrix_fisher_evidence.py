"""MatrixFisherRotationEvidence and PlanarTranslationEvidence
(archive/legacy_operators/matrix_fisher_evidence.py:55-671) on the GPU."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import numpy as np

from .. import _abi
from ..belief import BeliefGaussianInfo
from ..certificates import (CertBundle, ConditioningCert, ExpectedEffect, InfluenceCert, MismatchCert)
from ..constants import GC_EPS_LIFT, GC_EPS_MASS, GC_EPS_PSD


@dataclass
class ScatterMetrics:
    eigenvalues: np.ndarray   # (3,) descending
    eigenvectors: np.ndarray  # (3, 3) columns
    linearity: float
    planarity: float
    sphericity: float
    anisotropy: float
    effective_rank: float


@dataclass
class MatrixFisherResult:
    R_mf: np.ndarray
    L_rot: np.ndarray
    h_rot: np.ndarray
    delta_rot: np.ndarray
    svd_singular_values: np.ndarray
    map_scatter_metrics: ScatterMetrics
    scan_scatter_metrics: ScatterMetrics


@dataclass
class PlanarTranslationResult:
    t_wls: np.ndarray
    L_trans: np.ndarray
    h_trans: np.ndarray
    delta_trans: np.ndarray
    xy_info_scale: float
    z_info_scale: float


def _scatter(v) -> ScatterMetrics:
    return ScatterMetrics(eigenvalues=v[0:3].copy(), eigenvectors=v[3:12].reshape(3, 3).copy(),
                          linearity=float(v[12]), planarity=float(v[13]), sphericity=float(v[14]),
                          anisotropy=float(v[15]), effective_rank=float(v[16]))


def _dev(ctx, *arrays):
    """The operands in one packed upload (None stays None)."""
    idx = [i for i, a in enumerate(arrays) if a is not None]
    up = _abi.upload_many(ctx, [arrays[i] for i in idx])
    out = [None] * len(arrays)
    for i, d in zip(idx, up):
        out[i] = d
    return out


def matrix_fisher_batch(pose_pred, scan_s_dir, scan_N, scan_S_dir_scatter, map_S_dir, map_N_dir, map_S_dir_scatter,
                        eps_psd=GC_EPS_PSD, eps_mass=GC_EPS_MASS, ctx=None):
    """H predicted poses (H,6) x per-hypothesis scan bins (H,B,*) against one map (B,*) ->
    (H, GC_MF_OUT) records (include/gcslam.h)."""
    ctx = ctx or _abi.default_context()
    pose = np.asarray(pose_pred, np.float64).reshape(-1, 6)
    H = pose.shape[0]
    sN = np.asarray(scan_N, np.float64).reshape(H, -1)
    B = sN.shape[1]
    if not 1 <= B <= 64:
        raise ValueError(f"bin count must be in [1, 64], got {B}")
    d = _dev(ctx, pose, np.asarray(scan_s_dir).reshape(H, B, 3), sN,
             None if scan_S_dir_scatter is None else np.asarray(scan_S_dir_scatter).reshape(H, B, 9),
             np.asarray(map_S_dir).reshape(B, 3), np.asarray(map_N_dir).reshape(B),
             None if map_S_dir_scatter is None else np.asarray(map_S_dir_scatter).reshape(B, 9))
    out = _abi.DeviceArray(ctx, (H, _abi.GC_MF_OUT))
    _abi.call("gc_matrix_fisher_batch", ctx.handle, H, B, *[x.ptr if x is not None else None for x in d],
              float(eps_psd), float(eps_mass), out.ptr, ctx=ctx)
    return out.download()


def matrix_fisher_rotation_evidence(belief_pred: BeliefGaussianInfo, scan_s_dir, scan_S_dir_scatter, scan_N,
                                    map_S_dir, map_S_dir_scatter, map_N_dir, eps_psd: float = GC_EPS_PSD,
                                    eps_lift: float = GC_EPS_LIFT, eps_mass: float = GC_EPS_MASS, ctx=None
                                    ) -> Tuple[MatrixFisherResult, CertBundle, ExpectedEffect]:
    pose = belief_pred.world_pose(eps_lift, ctx)[None]
    o = matrix_fisher_batch(pose, np.asarray(scan_s_dir)[None], np.asarray(scan_N)[None],
                            np.asarray(scan_S_dir_scatter)[None], map_S_dir, map_N_dir, map_S_dir_scatter, eps_psd,
                            eps_mass, ctx)[0]
    svd = o[24:27].copy()
    N_eff = float(o[27])
    res = MatrixFisherResult(R_mf=o[0:9].reshape(3, 3).copy(), L_rot=o[9:18].reshape(3, 3).copy(),
                             h_rot=o[18:21].copy(), delta_rot=o[21:24].copy(), svd_singular_values=svd,
                             map_scatter_metrics=_scatter(o[32:49]), scan_scatter_metrics=_scatter(o[49:66]))
    ev = np.sort(np.array([svd[1] + svd[2], svd[0] + svd[2], svd[0] + svd[1]]))
    eig_min, eig_max = float(max(ev[0], eps_psd)), float(max(ev[2], eps_psd))
    cert = CertBundle.create_approx(
        chart_id=belief_pred.chart_id, anchor_id=belief_pred.anchor_id, triggers=["MatrixFisherRotationEvidence"],
        conditioning=ConditioningCert(eig_min=eig_min, eig_max=eig_max, cond=eig_max / (eig_min + eps_mass),
                                      near_null_count=int(np.sum(svd < eps_mass))),
        mismatch=MismatchCert(nll_per_ess=float(o[28]), directional_score=float(np.sum(svd))),
        influence=InfluenceCert(lift_strength=0.0, psd_projection_delta=float(o[29]),
                                mass_epsilon_ratio=float(eps_mass / (N_eff + eps_mass)), anchor_drift_rho=0.0,
                                dt_scale=1.0, extrinsic_scale=1.0, trust_alpha=1.0))
    return res, cert, ExpectedEffect(objective_name="predicted_rotation_nll", predicted=float(o[31]))


def planar_translation_batch(pose_pred, R_hat, scan_p_bar, scan_Sigma_p, scan_N, map_centroid, map_Sigma_c,
                             map_N_pos, map_S_dir_scatter, map_N_dir, eps_psd=GC_EPS_PSD, eps_mass=GC_EPS_MASS,
                             ctx=None):
    """-> (H, GC_PT_OUT) records (include/gcslam.h)."""
    ctx = ctx or _abi.default_context()
    pose = np.asarray(pose_pred, np.float64).reshape(-1, 6)
    H = pose.shape[0]
    sN = np.asarray(scan_N, np.float64).reshape(H, -1)
    B = sN.shape[1]
    if not 1 <= B <= 64:
        raise ValueError(f"bin count must be in [1, 64], got {B}")
    d = _dev(ctx, pose, np.asarray(R_hat).reshape(H, 9), np.asarray(scan_p_bar).reshape(H, B, 3),
             np.asarray(scan_Sigma_p).reshape(H, B, 9), sN, np.asarray(map_centroid).reshape(B, 3),
             np.asarray(map_Sigma_c).reshape(B, 9), np.asarray(map_N_pos).reshape(B),
             np.asarray(map_S_dir_scatter).reshape(B, 9), np.asarray(map_N_dir).reshape(B))
    out = _abi.DeviceArray(ctx, (H, _abi.GC_PT_OUT))
    _abi.call("gc_planar_translation_batch", ctx.handle, H, B, *[x.ptr for x in d], float(eps_psd), float(eps_mass),
              out.ptr, ctx=ctx)
    return out.download()


def planar_translation_evidence(belief_pred: BeliefGaussianInfo, scan_p_bar, scan_Sigma_p, scan_N, map_centroid,
                                map_Sigma_c, map_N_pos, map_S_dir_scatter, map_N_dir, R_hat,
                                eps_psd: float = GC_EPS_PSD, eps_lift: float = GC_EPS_LIFT,
                                eps_mass: float = GC_EPS_MASS, ctx=None
                                ) -> Tuple[PlanarTranslationResult, CertBundle, ExpectedEffect]:
    pose = belief_pred.world_pose(eps_lift, ctx)[None]
    o = planar_translation_batch(pose, np.asarray(R_hat)[None], np.asarray(scan_p_bar)[None],
                                 np.asarray(scan_Sigma_p)[None], np.asarray(scan_N)[None], map_centroid, map_Sigma_c,
                                 map_N_pos, map_S_dir_scatter, map_N_dir, eps_psd, eps_mass, ctx)[0]
    N_eff = float(o[19])
    res = PlanarTranslationResult(t_wls=o[0:3].copy(), L_trans=o[3:12].reshape(3, 3).copy(), h_trans=o[12:15].copy(),
                                  delta_trans=o[15:18].copy(), xy_info_scale=float(o[23]), z_info_scale=float(o[24]))
    cert = CertBundle.create_approx(
        chart_id=belief_pred.chart_id, anchor_id=belief_pred.anchor_id, triggers=["PlanarTranslationEvidence"],
        mismatch=MismatchCert(nll_per_ess=float(o[20]), directional_score=float(o[18])),
        influence=InfluenceCert(psd_projection_delta=float(o[21]),
                                mass_epsilon_ratio=float(eps_mass / (N_eff + eps_mass))))
    return res, cert, ExpectedEffect(objective_name="predicted_translation_nll", predicted=float(o[25]))
