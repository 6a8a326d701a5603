"""KappaFromResultant (backend/operators/kappa.py:130-169) on the GPU."""

from __future__ import annotations

import numpy as np

from .. import _abi
from ..constants import GC_EPS_R, GC_KAPPA_BLEND_R0, GC_KAPPA_BLEND_TAU


def kappa_from_resultant_batch(R_bar, eps_r: float = GC_EPS_R, d: int = 3,
                               r0: float = GC_KAPPA_BLEND_R0, tau: float = GC_KAPPA_BLEND_TAU, ctx=None):
    ctx = ctx or _abi.default_context()
    R = np.ascontiguousarray(R_bar, dtype=np.float64)
    shape = R.shape
    R = R.reshape(-1)
    if R.size == 0:
        return R.reshape(shape)
    dr = _abi.DeviceArray.from_host(ctx, R)
    dk = _abi.DeviceArray(ctx, R.shape[0])
    _abi.call("gc_kappa_from_resultant_batch", ctx.handle, R.shape[0], dr.ptr, float(eps_r), float(d),
              float(r0), float(tau), dk.ptr, ctx=ctx)
    return dk.download().reshape(shape)
