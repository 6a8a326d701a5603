"""PoseUpdateFrobeniusRecompose (backend/operators/recompose.py:36-205) and AnchorDriftUpdate
(backend/operators/anchor_drift.py:50-191) on the GPU."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import numpy as np

from .. import _abi
from ..belief import BeliefGaussianInfo, stack
from ..certificates import CertBundle, ExpectedEffect, InfluenceCert
from ..constants import D_Z, GC_C_FROB, GC_EPS_LIFT, GC_EPS_PSD


@dataclass
class RecomposeResult:
    delta_pose: np.ndarray
    X_new: np.ndarray
    frobenius_strength: float
    bch_correction: np.ndarray


@dataclass
class AnchorDriftResult:
    rho: float
    drift_m: float
    drift_r: float
    new_anchor_id: str


def _run(name, X, z, L, h, extra, ctx, res_w):
    ctx = ctx or _abi.default_context()
    H = X.shape[0]
    d = _abi.upload_many(ctx, (X, z, L, h))
    oX, oz, oh, res = _abi.alloc_many(ctx, [(H, 6), (H, D_Z), (H, D_Z), (H, res_w)])
    if name == "gc_recompose_batch":
        dT = _abi.DeviceArray.from_host(ctx, np.ascontiguousarray(extra[0], np.float64).reshape(H))
        _abi.call(name, ctx.handle, H, *[x.ptr for x in d], dT.ptr, float(extra[1]), float(extra[2]), oX.ptr, oz.ptr,
                  oh.ptr, res.ptr, ctx=ctx)
    else:
        _abi.call(name, ctx.handle, H, *[x.ptr for x in d], float(extra[0]), oX.ptr, oz.ptr, oh.ptr, res.ptr, ctx=ctx)
    return tuple(_abi.download_many([oX, oz, oh, res]))


def recompose_batch(X, z, L, h, T, c_frob=GC_C_FROB, eps_lift=GC_EPS_LIFT, ctx=None):
    """-> X_new (H,6), z' (H,22), h' (H,22), res (H,19) = [δ' 6, X_new 6, s, bch 6]."""
    return _run("gc_recompose_batch", *(np.ascontiguousarray(a, np.float64) for a in (X, z, L, h)),
                (T, c_frob, eps_lift), ctx, _abi.GC_RECOMPOSE_OUT)


def anchor_drift_batch(X, z, L, h, eps_lift=GC_EPS_LIFT, ctx=None):
    """-> X' (H,6), z' (H,22), h' (H,22), res (H,3) = [ρ, drift_m, drift_r]."""
    return _run("gc_anchor_drift_batch", *(np.ascontiguousarray(a, np.float64) for a in (X, z, L, h)), (eps_lift,),
                ctx, _abi.GC_DRIFT_OUT)


def pose_update_frobenius_recompose(belief_post: BeliefGaussianInfo, total_trigger_magnitude: float,
                                    c_frob: float = GC_C_FROB, eps_lift: float = GC_EPS_LIFT, ctx=None
                                    ) -> Tuple[RecomposeResult, BeliefGaussianInfo, CertBundle, ExpectedEffect]:
    X, z, L, h = stack([belief_post])
    Xn, zn, hn, r = recompose_batch(X, z, L, h, [float(total_trigger_magnitude)], c_frob, eps_lift, ctx)
    r = r[0]
    s = float(r[12])
    res = RecomposeResult(delta_pose=r[0:6].copy(), X_new=r[6:12].copy(), frobenius_strength=s,
                          bch_correction=r[13:19].copy())
    cert = CertBundle.create_approx(chart_id=belief_post.chart_id, anchor_id=belief_post.anchor_id,
                                    triggers=["PoseUpdateFrobeniusRecompose"],
                                    frobenius_applied=s > float(np.finfo(np.float64).eps),
                                    influence=InfluenceCert.identity())
    out = BeliefGaussianInfo(belief_post.chart_id, belief_post.anchor_id, Xn[0], belief_post.stamp_sec, zn[0],
                             belief_post.L, hn[0], cert)
    return res, out, cert, ExpectedEffect(objective_name="predicted_pose_increment_magnitude",
                                          predicted=float(np.linalg.norm(res.delta_pose)))


def anchor_drift_update(belief: BeliefGaussianInfo, eps_lift: float = GC_EPS_LIFT, eps_psd: float = GC_EPS_PSD,
                        ctx=None) -> Tuple[AnchorDriftResult, BeliefGaussianInfo, CertBundle, ExpectedEffect]:
    X, z, L, h = stack([belief])
    Xn, zn, hn, r = anchor_drift_batch(X, z, L, h, eps_lift, ctx)
    rho = float(r[0, 0])
    new_id = f"anchor_{int(belief.stamp_sec * 1000) % 10000}"  # anchor_drift.py:147-149
    res = AnchorDriftResult(rho=rho, drift_m=float(r[0, 1]), drift_r=float(r[0, 2]), new_anchor_id=new_id)
    cert = CertBundle.create_approx(chart_id=belief.chart_id, anchor_id=new_id, triggers=["AnchorDriftUpdate"],
                                    influence=InfluenceCert.identity().with_overrides(anchor_drift_rho=rho))
    out = BeliefGaussianInfo(belief.chart_id, new_id, Xn[0], belief.stamp_sec, zn[0], belief.L, hn[0], cert)
    return res, out, cert, ExpectedEffect(objective_name="anchor_drift_rho", predicted=rho)
