"""PointBudgetResample (backend/operators/point_budget.py:31-221) on the GPU."""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Tuple

import numpy as np

from .. import _abi
from ..certificates import CertBundle, ExpectedEffect, InfluenceCert, SupportCert
from ..constants import GC_CHART_ID, GC_EPS_MASS, GC_N_POINTS_CAP


@dataclass
class PointBudgetResult:
    points: np.ndarray
    timestamps: np.ndarray
    weights: np.ndarray
    ring: np.ndarray
    tag: np.ndarray
    n_input: int
    n_output: int
    total_mass_in: float
    total_mass_out: float
    indices: np.ndarray = None  # selected source rows (-1 padded): the integer contract


def point_budget_resample(points, timestamps, weights, ring=None, tag=None,
                          n_points_cap: int = GC_N_POINTS_CAP, chart_id: str = GC_CHART_ID,
                          anchor_id: str = "initial", ctx=None
                          ) -> Tuple[PointBudgetResult, CertBundle, ExpectedEffect]:
    ctx = ctx or _abi.default_context()
    P = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
    n = P.shape[0]
    T = np.ascontiguousarray(timestamps, dtype=np.float64).reshape(-1)
    W = np.ascontiguousarray(weights, dtype=np.float64).reshape(-1)
    if T.shape[0] != n or W.shape[0] != n:
        raise ValueError(f"timestamps/weights must be ({n},), got {T.shape}, {W.shape}")
    if n == 0 or n_points_cap <= 0:
        raise ValueError("point_budget_resample needs n_input > 0 and n_points_cap > 0")
    RG = np.zeros(n, np.uint8) if ring is None else np.ascontiguousarray(ring, np.uint8).reshape(-1)
    TG = np.zeros(n, np.uint8) if tag is None else np.ascontiguousarray(tag, np.uint8).reshape(-1)
    cap = int(n_points_cap)
    dev = {k: _abi.DeviceArray.from_host(ctx, v, v.dtype) for k, v in
           dict(p=P, t=T, w=W, r=RG, g=TG).items()}
    out_p = _abi.DeviceArray(ctx, (cap, 3)); out_t = _abi.DeviceArray(ctx, cap)
    out_w = _abi.DeviceArray(ctx, cap); out_r = _abi.DeviceArray(ctx, cap, np.uint8)
    out_g = _abi.DeviceArray(ctx, cap, np.uint8); out_i = _abi.DeviceArray(ctx, cap, np.int64)
    scal = _abi.DeviceArray(ctx, 8)
    _abi.call("gc_point_budget_resample", ctx.handle, dev["p"].ptr, dev["t"].ptr, dev["w"].ptr,
              dev["r"].ptr, dev["g"].ptr, n, cap, out_p.ptr, out_t.ptr, out_w.ptr, out_r.ptr,
              out_g.ptr, out_i.ptr, scal.ptr, ctx=ctx)
    s = scal.download()
    mass_in = float(s[0])
    res = PointBudgetResult(points=out_p.download(), timestamps=out_t.download(), weights=out_w.download(),
                            ring=out_r.download(), tag=out_g.download(), n_input=n, n_output=int(s[5]),
                            total_mass_in=mass_in, total_mass_out=mass_in, indices=out_i.download())
    support_frac = min(1.0, cap / (n + GC_EPS_MASS))
    cert = CertBundle.create_approx(
        chart_id=chart_id, anchor_id=anchor_id, triggers=["PointBudgetResample"],
        support=SupportCert(ess_total=float(s[3]), support_frac=support_frac),
        influence=InfluenceCert.identity().with_overrides(
            mass_epsilon_ratio=GC_EPS_MASS / (mass_in + GC_EPS_MASS)))
    return res, cert, ExpectedEffect(objective_name="predicted_ess", predicted=float(s[3]))


def budget_stride(n_input: int, n_points_cap: int) -> int:
    """point_budget.py:160."""
    return max(1, int(math.ceil(n_input / n_points_cap)))
