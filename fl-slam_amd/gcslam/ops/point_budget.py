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


def _rows(x, width=None) -> int:
    sh = x.shape if isinstance(x, _abi.DeviceArray) else np.shape(x)
    n = int(np.prod(sh)) if sh else 1
    return n // width if width else n


def point_budget_resample(points, timestamps, weights, ring=None, tag=None,
                          n_points_cap: int = GC_N_POINTS_CAP, chart_id: str = GC_CHART_ID,
                          anchor_id: str = "initial", ctx=None, device_out: bool = False
                          ) -> Tuple[PointBudgetResult, CertBundle, ExpectedEffect]:
    """Host arrays or DeviceArrays in; with device_out the result's arrays stay in HBM (DeviceArray)."""
    ctx = ctx or _abi.default_context()
    n = _rows(points, 3)
    if _rows(timestamps) != n or _rows(weights) != n:
        raise ValueError(f"timestamps/weights must be ({n},), got {np.shape(timestamps)}, {np.shape(weights)}")
    if n == 0 or n_points_cap <= 0:
        raise ValueError("point_budget_resample needs n_input > 0 and n_points_cap > 0")
    cap = int(n_points_cap)
    dev = dict(p=_abi.device_input(ctx, points, np.float64, (n, 3)),
               t=_abi.device_input(ctx, timestamps, np.float64, (n,)),
               w=_abi.device_input(ctx, weights, np.float64, (n,)))
    for k, v in (("r", ring), ("g", tag)):
        if v is None:
            dev[k] = _abi.DeviceArray(ctx, n, np.uint8)
            dev[k].zero()
        else:
            dev[k] = _abi.device_input(ctx, v, np.uint8, (n,))
    out_p, out_t, out_w, out_r, out_g, out_i, scal = _abi.alloc_many(
        ctx, [(cap, 3), cap, cap, (cap, np.uint8), (cap, np.uint8), (cap, np.int64), 8])
    _abi.call("gc_point_budget_resample", ctx.handle, dev["p"].ptr, dev["t"].ptr, dev["w"].ptr,
              dev["r"].ptr, dev["g"].ptr, n, cap, out_p.ptr, out_t.ptr, out_w.ptr, out_r.ptr,
              out_g.ptr, out_i.ptr, scal.ptr, ctx=ctx)
    if device_out:
        s = scal.download()
        arr = (out_p, out_t, out_w, out_r, out_g, out_i)
    else:
        *arr, s = _abi.download_many([out_p, out_t, out_w, out_r, out_g, out_i, scal])
    mass_in = float(s[0])
    res = PointBudgetResult(points=arr[0], timestamps=arr[1], weights=arr[2], ring=arr[3], tag=arr[4], n_input=n,
                            n_output=int(s[5]), total_mass_in=mass_in, total_mass_out=mass_in, indices=arr[5])
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
