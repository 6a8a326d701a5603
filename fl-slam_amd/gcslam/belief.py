"""BeliefGaussianInfo (common/belief.py:197-460), field-compatible: the Gaussian belief on the
22-D augmented tangent chart in information form. ``mean_increment`` and ``world_pose`` run on
the GPU (gc_belief_world_pose_batch); there is no host solve."""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

from . import _abi
from .certificates import CertBundle, ConditioningCert
from .constants import D_Z, GC_CHART_ID, GC_EPS_LIFT


@dataclass
class BeliefGaussianInfo:
    chart_id: str
    anchor_id: str
    X_anchor: np.ndarray  # (6,) SE3 as [trans, rotvec]
    stamp_sec: float
    z_lin: np.ndarray     # (D_Z,)
    L: np.ndarray         # (D_Z, D_Z)
    h: np.ndarray         # (D_Z,)
    cert: CertBundle = field(default=None)

    def __post_init__(self):
        if self.chart_id != GC_CHART_ID:
            raise ValueError(f"Invalid chart_id: {self.chart_id}, expected {GC_CHART_ID}")
        self.X_anchor = np.asarray(self.X_anchor, dtype=np.float64).reshape(6)
        self.z_lin = np.asarray(self.z_lin, dtype=np.float64).reshape(D_Z)
        self.L = np.asarray(self.L, dtype=np.float64).reshape(D_Z, D_Z)
        self.h = np.asarray(self.h, dtype=np.float64).reshape(D_Z)
        if self.cert is None:
            self.cert = CertBundle.create_exact(chart_id=self.chart_id, anchor_id=self.anchor_id)

    @classmethod
    def create_identity_prior(cls, anchor_id: str, stamp_sec: float, prior_precision: float = 1e-6
                              ) -> "BeliefGaussianInfo":
        """belief.py:328-371."""
        cert = CertBundle.create_exact(chart_id=GC_CHART_ID, anchor_id=anchor_id,
                                       conditioning=ConditioningCert(eig_min=prior_precision, eig_max=prior_precision,
                                                                     cond=1.0, near_null_count=D_Z))
        return cls(GC_CHART_ID, anchor_id, np.zeros(6), float(stamp_sec), np.zeros(D_Z),
                   prior_precision * np.eye(D_Z), np.zeros(D_Z), cert)

    def _pose_and_mean(self, eps_lift: float, ctx):
        """(world pose, mean increment) from one launch, remembered for the belief's current (X, L, h, ε):
        the node asks a belief for both, several times per scan (the cache key is the arrays' bytes,
        so an in-place edit of X_anchor / L / h is seen)."""
        key = (float(eps_lift), self.X_anchor.tobytes(), self.L.tobytes(), self.h.tobytes())
        c = self.__dict__.get("_pm_cache")
        if c is None or c[0] != key:
            p, m = world_pose_batch([self], eps_lift, ctx)
            c = (key, p[0], m[0])
            self.__dict__["_pm_cache"] = c
        return c[1], c[2]

    def mean_increment(self, eps_lift: float = GC_EPS_LIFT, ctx=None) -> np.ndarray:
        """δz* = (L + eps_lift I)⁻¹ h (belief.py:373-386)."""
        return self._pose_and_mean(eps_lift, ctx)[1].copy()

    def world_pose(self, eps_lift: float = GC_EPS_LIFT, ctx=None) -> np.ndarray:
        """X_anchor ∘ Exp(δz*[0:6]) (belief.py:408-425)."""
        return self._pose_and_mean(eps_lift, ctx)[0].copy()


def stack(beliefs: List[BeliefGaussianInfo]) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """(X (H,6), z (H,22), L (H,22,22), h (H,22)) as contiguous f64."""
    X = np.ascontiguousarray(np.stack([b.X_anchor for b in beliefs]), dtype=np.float64)
    z = np.ascontiguousarray(np.stack([b.z_lin for b in beliefs]), dtype=np.float64)
    L = np.ascontiguousarray(np.stack([b.L for b in beliefs]), dtype=np.float64)
    h = np.ascontiguousarray(np.stack([b.h for b in beliefs]), dtype=np.float64)
    return X, z, L, h


def world_pose_batch(beliefs: List[BeliefGaussianInfo], eps_lift: float = GC_EPS_LIFT, ctx=None,
                     arrays: Optional[tuple] = None):
    """World poses (H,6) and mean increments (H,22) of H beliefs, one launch."""
    ctx = ctx or _abi.default_context()
    X, _, L, h = arrays if arrays is not None else stack(beliefs)
    H = X.shape[0]
    dX, dL, dh = _abi.upload_many(ctx, (X, L, h))
    dp, dm = _abi.alloc_many(ctx, [(H, 6), (H, D_Z)])
    _abi.call("gc_belief_world_pose_batch", ctx.handle, H, dX.ptr, dL.ptr, dh.ptr, float(eps_lift), dp.ptr, dm.ptr,
              ctx=ctx)
    return tuple(_abi.download_many([dp, dm]))
