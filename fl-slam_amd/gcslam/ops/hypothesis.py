"""HypothesisBarycenterProjection (backend/operators/hypothesis.py:40-236) on the GPU."""

from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple

import numpy as np

from .. import _abi
from ..belief import BeliefGaussianInfo, stack
from ..certificates import CertBundle, ConditioningCert, ExpectedEffect, InfluenceCert, SupportCert
from ..constants import D_Z, GC_CHART_ID, GC_EPS_LIFT, GC_EPS_PSD, GC_HYP_WEIGHT_FLOOR, GC_K_HYP


@dataclass
class HypothesisProjectionResult:
    belief_out: BeliefGaussianInfo
    floor_adjustment: float


def hypothesis_barycenter_batch(L, h, z, weights, floor, eps_psd=GC_EPS_PSD, eps_lift=GC_EPS_LIFT, ctx=None):
    """(K,22,22),(K,22),(K,22),(K,) -> L (PSD), h, z_lin, cert (16) (include/gcslam.h GC_BARY_CERT)."""
    ctx = ctx or _abi.default_context()
    Ls = np.ascontiguousarray(L, np.float64).reshape(-1, D_Z, D_Z)
    K = Ls.shape[0]
    d = _abi.upload_many(ctx, (Ls, np.ascontiguousarray(h, np.float64).reshape(K, D_Z),
                               np.ascontiguousarray(z, np.float64).reshape(K, D_Z),
                               np.ascontiguousarray(weights, np.float64).reshape(K)))
    oL, oh, oz, oc = _abi.alloc_many(ctx, [(D_Z, D_Z), D_Z, D_Z, _abi.GC_BARY_CERT])
    _abi.call("gc_hypothesis_barycenter", ctx.handle, K, *[x.ptr for x in d], float(floor), float(eps_psd),
              float(eps_lift), oL.ptr, oh.ptr, oz.ptr, oc.ptr, ctx=ctx)
    return tuple(_abi.download_many([oL, oh, oz, oc]))


def hypothesis_barycenter_projection(hypotheses: List[BeliefGaussianInfo], weights, K_HYP: int = GC_K_HYP,
                                     HYP_WEIGHT_FLOOR: float = GC_HYP_WEIGHT_FLOOR, eps_psd: float = GC_EPS_PSD,
                                     eps_lift: float = GC_EPS_LIFT, ctx=None
                                     ) -> Tuple[HypothesisProjectionResult, CertBundle, ExpectedEffect]:
    w = np.asarray(weights, dtype=np.float64)
    if len(hypotheses) != K_HYP:
        raise ValueError(f"Expected {K_HYP} hypotheses, got {len(hypotheses)}")
    if w.shape != (K_HYP,):
        raise ValueError(f"Expected weights shape ({K_HYP},), got {w.shape}")
    _, z, L, h = stack(hypotheses)
    Lo, ho, zo, c = hypothesis_barycenter_batch(L, h, z, w, HYP_WEIGHT_FLOOR, eps_psd, eps_lift, ctx)
    t = hypotheses[0]
    cert = CertBundle.create_approx(
        chart_id=GC_CHART_ID, anchor_id=t.anchor_id, triggers=["HypothesisProjection", "I-projection-info-barycenter"],
        conditioning=ConditioningCert(eig_min=float(c[7]), eig_max=float(c[8]), cond=float(c[9]),
                                      near_null_count=int(c[10])),
        support=SupportCert(ess_total=float(c[2]), support_frac=float(c[3])),
        influence=InfluenceCert.identity().with_overrides(psd_projection_delta=float(c[5]),
                                                          mass_epsilon_ratio=float(c[4])))
    out = BeliefGaussianInfo(GC_CHART_ID, t.anchor_id, t.X_anchor, t.stamp_sec, zo, Lo, ho, cert)
    return (HypothesisProjectionResult(belief_out=out, floor_adjustment=float(c[0])), cert,
            ExpectedEffect(objective_name="predicted_projection_spread_proxy", predicted=float(c[1])))
