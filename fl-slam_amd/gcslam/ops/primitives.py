"""DomainProjectionPSD (common/primitives.py:80-123, :310-359) on the GPU."""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .. import _abi
from ..constants import GC_EPS_LIFT, GC_EPS_PSD


@dataclass
class ConditioningInfo:
    eig_min: float
    eig_max: float
    cond: float
    near_null_count: int


@dataclass
class DomainProjectionPSDResult:
    M_psd: np.ndarray
    projection_delta: float
    sym_delta: float
    conditioning: ConditioningInfo


def domain_projection_psd_batch(M, eps_psd: float = GC_EPS_PSD, ctx=None):
    """(batch, d, d) -> (M_psd (batch, d, d), cert (batch, 6))."""
    ctx = ctx or _abi.default_context()
    A = np.ascontiguousarray(M, dtype=np.float64)
    if A.ndim != 3 or A.shape[1] != A.shape[2]:
        raise ValueError(f"expected (batch, d, d), got {A.shape}")
    b, d, _ = A.shape
    dm = _abi.DeviceArray.from_host(ctx, A)
    do, dc = _abi.alloc_many(ctx, [A.shape, (b, 6)])
    _abi.call("gc_domain_projection_psd_batch", ctx.handle, b, d, dm.ptr, float(eps_psd), do.ptr, dc.ptr, ctx=ctx)
    return tuple(_abi.download_many([do, dc]))


def spd_cholesky_inverse_lifted(L, eps_lift: float = GC_EPS_LIFT, ctx=None, device_out: bool = False):
    """spd_cholesky_inverse_lifted_core (common/primitives.py:169-192): ((L + eps_lift I)⁻¹, lift) for
    an n x n (or a batch (b, n, n)) SPD matrix, n <= 22, host or DeviceArray in."""
    ctx = ctx or _abi.default_context()
    sh = L.shape if isinstance(L, _abi.DeviceArray) else np.shape(L)
    n = sh[-1]
    b = int(np.prod(sh[:-2])) if len(sh) > 2 else 1
    dL = _abi.device_input(ctx, L, np.float64, (b, n, n))
    out = _abi.DeviceArray(ctx, (b, n, n))
    _abi.call("gc_spd_inverse_lifted_batch", ctx.handle, b, n, dL.ptr, float(eps_lift), out.ptr, ctx=ctx)
    res = out.view(sh) if device_out else out.download().reshape(sh)
    return res, float(eps_lift) * n


def domain_projection_psd(M, eps_psd: float = GC_EPS_PSD, ctx=None) -> DomainProjectionPSDResult:
    Mp, c = domain_projection_psd_batch(np.asarray(M, dtype=np.float64)[None], eps_psd, ctx)
    c = c[0]
    return DomainProjectionPSDResult(M_psd=Mp[0], projection_delta=float(c[0]), sym_delta=float(c[1]),
                                     conditioning=ConditioningInfo(float(c[2]), float(c[3]), float(c[4]),
                                                                   int(c[5])))
