"""FusionScaleFromCertificates and InfoFusionAdditive (backend/operators/fusion.py:36-230) on the GPU."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import numpy as np

from .. import _abi
from ..belief import BeliefGaussianInfo, stack
from ..certificates import (CertBundle, ConditioningCert, ExpectedEffect, InfluenceCert, OverconfidenceCert)
from ..constants import (D_Z, GC_ALPHA_MAX, GC_ALPHA_MIN, GC_C0_COND, GC_CHART_ID, GC_EPS_MASS, GC_EPS_PSD,
                         GC_KAPPA_SCALE)


@dataclass
class FusionScaleResult:
    alpha: float


def fusion_scale_batch(rows, alpha_min=GC_ALPHA_MIN, alpha_max=GC_ALPHA_MAX, c0_cond=GC_C0_COND, ctx=None):
    """rows (H, 8) = [cond, ess_total, support_frac, excitation_total, dt_asymmetry, z_to_xy_ratio,
    power_beta, nll_per_ess] -> (H, 4) = [alpha, excitation_total, ess_to_excitation, cond_to_support]."""
    ctx = ctx or _abi.default_context()
    R = np.ascontiguousarray(rows, np.float64).reshape(-1, _abi.GC_FUSION_ROW)
    H = R.shape[0]
    dr, do = _abi.DeviceArray.from_host(ctx, R), _abi.DeviceArray(ctx, (H, _abi.GC_FUSION_OUT))
    _abi.call("gc_fusion_scale_batch", ctx.handle, H, dr.ptr, float(alpha_min), float(alpha_max), float(c0_cond),
              GC_EPS_MASS, do.ptr, ctx=ctx)
    return do.download()


def fusion_scale_from_certificates(cert_evidence: CertBundle, cert_belief: CertBundle,
                                   alpha_min: float = GC_ALPHA_MIN, alpha_max: float = GC_ALPHA_MAX,
                                   kappa_scale: float = GC_KAPPA_SCALE, c0_cond: float = GC_C0_COND,
                                   chart_id: str = GC_CHART_ID, anchor_id: str = "initial", ctx=None
                                   ) -> Tuple[FusionScaleResult, CertBundle, ExpectedEffect]:
    ce = cert_evidence
    row = [ce.conditioning.cond, ce.support.ess_total, ce.support.support_frac,
           ce.excitation.dt_effect + ce.excitation.extrinsic_effect, ce.overconfidence.dt_asymmetry,
           ce.overconfidence.z_to_xy_ratio, ce.influence.power_beta, ce.mismatch.nll_per_ess]
    o = fusion_scale_batch([row], alpha_min, alpha_max, c0_cond, ctx)[0]
    alpha = float(o[0])
    cert = CertBundle.create_exact(
        chart_id=chart_id, anchor_id=anchor_id,
        overconfidence=OverconfidenceCert(excitation_total=float(o[1]), ess_to_excitation=float(o[2]),
                                          cond_to_support=float(o[3]), dt_asymmetry=float(row[4]),
                                          z_to_xy_ratio=float(row[5])),
        influence=InfluenceCert.identity().with_overrides(trust_alpha=alpha))
    return FusionScaleResult(alpha=alpha), cert, ExpectedEffect(objective_name="fusion_alpha", predicted=alpha)


def info_fusion_additive_batch(L_pred, h_pred, L_evidence, h_evidence, alpha, eps_psd=GC_EPS_PSD, ctx=None):
    """(H,22,22) ... alpha (H,) -> L_post (PSD), h_post, cert (H,6) PSD certificate."""
    ctx = ctx or _abi.default_context()
    Lp = np.ascontiguousarray(L_pred, np.float64).reshape(-1, D_Z, D_Z)
    H = Lp.shape[0]
    hp = np.ascontiguousarray(h_pred, np.float64).reshape(H, D_Z)
    Le = np.ascontiguousarray(L_evidence, np.float64).reshape(H, D_Z, D_Z)
    he = np.ascontiguousarray(h_evidence, np.float64).reshape(H, D_Z)
    al = np.ascontiguousarray(np.broadcast_to(np.asarray(alpha, np.float64).reshape(-1), (H,)))
    d = _abi.upload_many(ctx, (Lp, hp, Le, he, al))
    Lo, ho, co = _abi.alloc_many(ctx, [Lp.shape, hp.shape, (H, 6)])
    _abi.call("gc_info_fusion_additive_batch", ctx.handle, H, *[x.ptr for x in d], float(eps_psd), Lo.ptr, ho.ptr,
              co.ptr, ctx=ctx)
    return tuple(_abi.download_many([Lo, ho, co]))


def info_fusion_additive(belief_pred: BeliefGaussianInfo, L_evidence, h_evidence, alpha: float,
                         eps_psd: float = GC_EPS_PSD, chart_id: str = GC_CHART_ID, anchor_id: str = "initial",
                         ctx=None) -> Tuple[BeliefGaussianInfo, CertBundle, ExpectedEffect]:
    _, _, L, h = stack([belief_pred])
    Lo, ho, c = info_fusion_additive_batch(L, h, np.asarray(L_evidence)[None], np.asarray(h_evidence)[None],
                                           [float(alpha)], eps_psd, ctx)
    c = c[0]
    cert = CertBundle.create_approx(
        chart_id=chart_id, anchor_id=anchor_id, triggers=["InfoFusionAdditive"],
        conditioning=ConditioningCert(eig_min=float(c[2]), eig_max=float(c[3]), cond=float(c[4]),
                                      near_null_count=int(c[5])),
        influence=InfluenceCert.identity().with_overrides(psd_projection_delta=float(c[0]), trust_alpha=float(alpha)))
    post = BeliefGaussianInfo(chart_id, anchor_id, belief_pred.X_anchor, belief_pred.stamp_sec, belief_pred.z_lin,
                              Lo[0], ho[0], cert)
    # trace increase from the two diagonals (expected-effect bookkeeping only)
    dtr = float(np.trace(Lo[0]) - np.trace(belief_pred.L))
    return post, cert, ExpectedEffect(objective_name="predicted_info_trace_increase", predicted=dtr)
