"""Excitation prior scaling (backend/operators/excitation.py:14-64) on the GPU."""

from __future__ import annotations

import numpy as np

from .. import _abi
from ..constants import D_Z, GC_EXC_EPS


def excitation_scaling_batch(L_evidence, L_prior, h_prior, eps=GC_EXC_EPS, ctx=None):
    """(H,22,22) evidence/prior -> (s (H,2) = [s_dt, s_ex], L_prior_scaled, h_prior_scaled)."""
    ctx = ctx or _abi.default_context()
    Le = np.ascontiguousarray(L_evidence, np.float64).reshape(-1, D_Z, D_Z)
    Lp = np.ascontiguousarray(L_prior, np.float64).reshape(-1, D_Z, D_Z)
    hp = np.ascontiguousarray(h_prior, np.float64).reshape(-1, D_Z)
    H = Le.shape[0]
    d = _abi.upload_many(ctx, (Le, Lp, hp))
    s, Lo, ho = _abi.alloc_many(ctx, [(H, 2), Lp.shape, hp.shape])
    _abi.call("gc_excitation_scaling_batch", ctx.handle, H, d[0].ptr, d[1].ptr, d[2].ptr, float(eps), s.ptr, Lo.ptr,
              ho.ptr, ctx=ctx)
    return tuple(_abi.download_many([s, Lo, ho]))


def compute_excitation_scales_jax(L_evidence, L_prior, eps: float = GC_EXC_EPS, ctx=None):
    """-> (s_dt, s_ex)."""
    s, _, _ = excitation_scaling_batch(L_evidence, L_prior, np.zeros(D_Z), eps, ctx)
    return float(s[0, 0]), float(s[0, 1])


def apply_excitation_prior_scaling_jax(L_prior, h_prior, s_dt, s_ex, ctx=None):
    """Prior rows/cols 15 scaled by (1 − s_dt), 16..21 by (1 − s_ex) -> (L_scaled, h_scaled)."""
    ctx = ctx or _abi.default_context()
    Lp = np.ascontiguousarray(L_prior, np.float64).reshape(1, D_Z, D_Z)
    hp = np.ascontiguousarray(h_prior, np.float64).reshape(1, D_Z)
    d = _abi.upload_many(ctx, (Lp, hp, np.array([[float(s_dt), float(s_ex)]])))
    Lo, ho = _abi.alloc_many(ctx, [Lp.shape, hp.shape])
    _abi.call("gc_excitation_scaling_batch", ctx.handle, 1, None, d[0].ptr, d[1].ptr, GC_EXC_EPS, d[2].ptr, Lo.ptr,
              ho.ptr, ctx=ctx)
    Lh, hh = _abi.download_many([Lo, ho])
    return Lh[0], hh[0]
