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


def deskew_batch(points, timestamps, weights, scan_start_time, scan_end_time, xi_batch, ctx=None):
    """H twists over one point set -> (points (H,N,3), weights (H,N), sum_w (H,))."""
    ctx = ctx or _abi.default_context()
    P = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
    n = P.shape[0]
    T = np.ascontiguousarray(timestamps, dtype=np.float64).reshape(-1)
    W = np.ascontiguousarray(weights, dtype=np.float64).reshape(-1)
    X = np.ascontiguousarray(xi_batch, dtype=np.float64).reshape(-1, 6)
    if T.shape[0] != n or W.shape[0] != n:
        raise ValueError("timestamps/weights must match points")
    H = X.shape[0]
    dp, dt, dw, dx = (_abi.DeviceArray.from_host(ctx, a) for a in (P, T, W, X))
    op = _abi.DeviceArray(ctx, (H, n, 3)); ow = _abi.DeviceArray(ctx, (H, n)); os_ = _abi.DeviceArray(ctx, H)
    _abi.call("gc_deskew_constant_twist", ctx.handle, H, n, dp.ptr, dt.ptr, dw.ptr,
              float(scan_start_time), float(scan_end_time), dx.ptr, op.ptr, ow.ptr, os_.ptr, ctx=ctx)
    return op.download(), ow.download(), os_.download()


def deskew_constant_twist(points, timestamps, weights, scan_start_time: float, scan_end_time: float,
                          xi_body, ess_imu: float, chart_id: str, anchor_id: str, ctx=None
                          ) -> Tuple[DeskewConstantTwistResult, CertBundle, ExpectedEffect]:
    pts, w_out, sw = deskew_batch(points, timestamps, weights, scan_start_time, scan_end_time,
                                  np.asarray(xi_body, dtype=np.float64).reshape(1, 6), ctx)
    w_in = np.asarray(weights, dtype=np.float64).reshape(-1)
    # retained = Σ w_out / (Σ w_in + ε)  (deskew_constant_twist.py:104)
    retained = float(sw[0] / (np.sum(w_in) + GC_EPS_MASS))
    res = DeskewConstantTwistResult(points=pts[0], timestamps=np.asarray(timestamps, np.float64),
                                    weights=w_out[0], ess_imu=float(ess_imu))
    cert = CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id,
                                   support=SupportCert(ess_total=float(ess_imu), support_frac=retained),
                                   influence=InfluenceCert.identity())
    return res, cert, ExpectedEffect(objective_name="deskew_variance_reduction_proxy", predicted=0.0)
