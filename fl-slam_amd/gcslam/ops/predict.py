"""PredictDiffusion (backend/operators/predict.py:43-214) on the GPU."""

from __future__ import annotations

from typing import Tuple

import numpy as np

from .. import _abi
from ..belief import BeliefGaussianInfo, stack
from ..certificates import CertBundle, ConditioningCert, ExpectedEffect, InfluenceCert
from ..constants import D_Z, GC_EPS_LIFT, GC_EPS_PSD, GC_OU_DAMPING_LAMBDA


def predict_diffusion_batch(L, h, Q, dt_sec, eps_psd=GC_EPS_PSD, eps_lift=GC_EPS_LIFT,
                            lambda_ou=GC_OU_DAMPING_LAMBDA, ctx=None):
    """(H,22,22), (H,22) -> L_pred, h_pred, cert (H, 8) = [lift, psd Δ, eig_min, eig_max, cond, nnc,
    trace Σ', trigger]."""
    ctx = ctx or _abi.default_context()
    L = np.ascontiguousarray(L, dtype=np.float64).reshape(-1, D_Z, D_Z)
    h = np.ascontiguousarray(h, dtype=np.float64).reshape(-1, D_Z)
    Qa = np.ascontiguousarray(Q, dtype=np.float64)
    if Qa.shape != (D_Z, D_Z):
        raise ValueError(f"Q must be ({D_Z}, {D_Z}), got {Qa.shape}")
    H = L.shape[0]
    dL, dh, dQ = _abi.upload_many(ctx, (L, h, Qa))
    oL, oh, oc = _abi.alloc_many(ctx, [L.shape, h.shape, (H, 8)])
    _abi.call("gc_predict_diffusion_batch", ctx.handle, H, dL.ptr, dh.ptr, dQ.ptr, float(dt_sec), float(eps_psd),
              float(eps_lift), float(lambda_ou), oL.ptr, oh.ptr, oc.ptr, ctx=ctx)
    return tuple(_abi.download_many([oL, oh, oc]))


def predict_diffusion(belief_prev: BeliefGaussianInfo, Q, dt_sec: float, eps_psd: float = GC_EPS_PSD,
                      eps_lift: float = GC_EPS_LIFT, lambda_ou: float = GC_OU_DAMPING_LAMBDA, ctx=None
                      ) -> Tuple[BeliefGaussianInfo, CertBundle, ExpectedEffect]:
    _, _, L, h = stack([belief_prev])
    Lp, hp, c = predict_diffusion_batch(L, h, Q, dt_sec, eps_psd, eps_lift, lambda_ou, ctx)
    c = c[0]
    cert = CertBundle.create_approx(
        chart_id=belief_prev.chart_id, anchor_id=belief_prev.anchor_id, triggers=["PredictDiffusion"],
        conditioning=ConditioningCert(eig_min=float(c[2]), eig_max=float(c[3]), cond=float(c[4]),
                                      near_null_count=int(c[5])),
        influence=InfluenceCert.identity().with_overrides(lift_strength=float(c[0]), psd_projection_delta=float(c[1]),
                                                          dt_scale=float(dt_sec)))
    out = BeliefGaussianInfo(belief_prev.chart_id, belief_prev.anchor_id, belief_prev.X_anchor,
                             belief_prev.stamp_sec + float(dt_sec), belief_prev.z_lin, Lp[0], hp[0], cert)
    return out, cert, ExpectedEffect(objective_name="predicted_cov_trace", predicted=float(c[6]))
