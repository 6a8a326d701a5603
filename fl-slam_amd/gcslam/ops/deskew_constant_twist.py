"""DeskewConstantTwist (backend/operators/deskew_constant_twist.py:23-117) on the GPU."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import numpy as np

from .. import _abi
from ..certificates import CertBundle, ExpectedEffect, InfluenceCert, SupportCert
from ..constants import GC_EPS_MASS


@dataclass
class DeskewConstantTwistResult:
    points: np.ndarray
    timestamps: np.ndarray
    weights: np.ndarray
    ess_imu: float


def _rows(x, width=1) -> int:
    sh = x.shape if isinstance(x, _abi.DeviceArray) else np.shape(x)
    return (int(np.prod(sh)) if sh else 1) // width


def deskew_batch(points, timestamps, weights, scan_start_time, scan_end_time, xi_batch, ctx=None,
                 device_out: bool = False):
    """H twists over one point set -> (points (H,N,3), weights (H,N), sum_w (H,)); inputs host or
    DeviceArray, the point arrays returned as DeviceArrays with device_out."""
    ctx = ctx or _abi.default_context()
    n = _rows(points, 3)
    if _rows(timestamps) != n or _rows(weights) != n:
        raise ValueError("timestamps/weights must match points")
    X = np.ascontiguousarray(xi_batch, dtype=np.float64).reshape(-1, 6)
    H = X.shape[0]
    dp = _abi.device_input(ctx, points, np.float64, (n, 3))
    dt = _abi.device_input(ctx, timestamps, np.float64, (n,))
    dw = _abi.device_input(ctx, weights, np.float64, (n,))
    dx = _abi.DeviceArray.from_host(ctx, X)
    op, ow, os_ = _abi.alloc_many(ctx, [(H, n, 3), (H, n), H])
    _abi.call("gc_deskew_constant_twist", ctx.handle, H, n, dp.ptr, dt.ptr, dw.ptr,
              float(scan_start_time), float(scan_end_time), dx.ptr, op.ptr, ow.ptr, os_.ptr, ctx=ctx)
    if device_out:
        return op, ow, os_.download()
    return tuple(_abi.download_many([op, ow, os_]))


def _weight_sum(ctx, weights) -> float:
    """Σ w_in: on the device for a DeviceArray (gc_budget_stats' mass_in, no round trip of w)."""
    if not isinstance(weights, _abi.DeviceArray):
        return float(np.sum(np.asarray(weights, dtype=np.float64).reshape(-1)))
    n = _rows(weights)
    scal = _abi.DeviceArray(ctx, 8)
    _abi.call("gc_budget_stats", ctx.handle, _abi.device_input(ctx, weights, np.float64, (n,)).ptr, n, n, scal.ptr,
              ctx=ctx)
    return float(scal.download()[0])


def deskew_constant_twist(points, timestamps, weights, scan_start_time: float, scan_end_time: float,
                          xi_body, ess_imu: float, chart_id: str, anchor_id: str, ctx=None,
                          device_out: bool = False
                          ) -> Tuple[DeskewConstantTwistResult, CertBundle, ExpectedEffect]:
    """Host arrays or DeviceArrays in; with device_out the deskewed points / weights stay in HBM."""
    ctx = ctx or _abi.default_context()
    pts, w_out, sw = deskew_batch(points, timestamps, weights, scan_start_time, scan_end_time,
                                  np.asarray(xi_body, dtype=np.float64).reshape(1, 6), ctx, device_out)
    # retained = Σ w_out / (Σ w_in + ε)  (deskew_constant_twist.py:104)
    retained = float(sw[0] / (_weight_sum(ctx, weights) + GC_EPS_MASS))
    n = _rows(points, 3)
    if device_out:
        res = DeskewConstantTwistResult(points=pts.view((n, 3)), timestamps=timestamps, weights=w_out.view((n,)),
                                        ess_imu=float(ess_imu))
    else:
        res = DeskewConstantTwistResult(points=pts[0], timestamps=np.asarray(timestamps, np.float64),
                                        weights=w_out[0], ess_imu=float(ess_imu))
    cert = CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id,
                                   support=SupportCert(ess_total=float(ess_imu), support_frac=retained),
                                   influence=InfluenceCert.identity())
    return res, cert, ExpectedEffect(objective_name="deskew_variance_reduction_proxy", predicted=0.0)
