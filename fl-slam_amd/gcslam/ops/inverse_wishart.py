"""Process- and measurement-noise inverse-Wishart operators (backend/operators/
inverse_wishart_jax.py:28-185, measurement_noise_iw_jax.py:26-100) on the GPU. The state
containers mirror backend/structures/inverse_wishart_jax.py / measurement_noise_iw_jax.py."""

from __future__ import annotations

from dataclasses import dataclass, replace

import numpy as np

from .. import _abi
from ..constants import D_Z, GC_EPS_LIFT, GC_EPS_PSD


@dataclass
class ProcessNoiseIWState:
    nu: np.ndarray   # (7,)
    Psi: np.ndarray  # (7, 6, 6)


@dataclass
class MeasurementNoiseIWState:
    nu: np.ndarray   # (3,) [gyro, accel, lidar]
    Psi: np.ndarray  # (3, 3, 3)


def _f(a, shape):
    return np.ascontiguousarray(np.asarray(a, np.float64).reshape(shape))


def process_noise_iw_suffstats_batch(L_pred, h_pred, L_post, h_post, eps_lift=GC_EPS_LIFT, ctx=None):
    """(H,22,22)/(H,22) pairs -> dPsi (H,7,6,6), dnu (H,7)."""
    ctx = ctx or _abi.default_context()
    Lq = _f(L_pred, (-1, D_Z, D_Z))
    H = Lq.shape[0]
    d = _abi.upload_many(ctx, (Lq, _f(h_pred, (H, D_Z)), _f(L_post, (H, D_Z, D_Z)), _f(h_post, (H, D_Z))))
    dP, dn = _abi.alloc_many(ctx, [(H, 7, 6, 6), (H, 7)])
    _abi.call("gc_iw_process_suffstats_batch", ctx.handle, H, *[x.ptr for x in d], float(eps_lift), dP.ptr, dn.ptr,
              ctx=ctx)
    return tuple(_abi.download_many([dP, dn]))


def process_noise_iw_suffstats_from_info_jax(L_pred, h_pred, L_post, h_post, eps_lift: float = GC_EPS_LIFT, ctx=None):
    dP, dn = process_noise_iw_suffstats_batch(L_pred, h_pred, L_post, h_post, eps_lift, ctx)
    return dP[0], dn[0]


def process_noise_iw_apply_suffstats_jax(pn_state: ProcessNoiseIWState, dPsi, dnu, dt_sec: float = 0.0,
                                         eps_psd: float = GC_EPS_PSD, nu_max: float = 1000.0, ctx=None):
    """-> (ProcessNoiseIWState, cert (2,) = [psd Δ sum, ν projection sum]). dt_sec unused (API compat)."""
    ctx = ctx or _abi.default_context()
    d = _abi.upload_many(ctx, (_f(pn_state.nu, 7), _f(pn_state.Psi, (7, 6, 6)), _f(dPsi, (7, 6, 6)), _f(dnu, 7)))
    on, oP, oc = _abi.alloc_many(ctx, [7, (7, 6, 6), 2])
    _abi.call("gc_iw_process_apply", ctx.handle, *[x.ptr for x in d], float(eps_psd), float(nu_max), on.ptr, oP.ptr,
              oc.ptr, ctx=ctx)
    nu, Psi, c = _abi.download_many([on, oP, oc])
    return replace(pn_state, nu=nu, Psi=Psi), c


def process_noise_state_to_Q_jax(pn_state: ProcessNoiseIWState, eps_psd: float = GC_EPS_PSD, ctx=None):
    """Q (22,22) = PSD(block-diag(Ψ_b / softplus⁺(ν_b − d_b − 1)))."""
    ctx = ctx or _abi.default_context()
    dn, dP = _abi.upload_many(ctx, (_f(pn_state.nu, 7), _f(pn_state.Psi, (7, 6, 6))))
    oQ = _abi.DeviceArray(ctx, (D_Z, D_Z))
    _abi.call("gc_iw_process_Q", ctx.handle, dn.ptr, dP.ptr, float(eps_psd), oQ.ptr, ctx=ctx)
    return oQ.download()


def measurement_noise_apply_suffstats_jax(mn_state: MeasurementNoiseIWState, dPsi, dnu, eps_psd: float = GC_EPS_PSD,
                                          nu_max: float = 1000.0, ctx=None):
    """-> (MeasurementNoiseIWState, cert (2,))."""
    ctx = ctx or _abi.default_context()
    d = _abi.upload_many(ctx, (_f(mn_state.nu, 3), _f(mn_state.Psi, (3, 3, 3)), _f(dPsi, (3, 3, 3)), _f(dnu, 3)))
    on, oP, oc = _abi.alloc_many(ctx, [3, (3, 3, 3), 2])
    _abi.call("gc_iw_meas_apply", ctx.handle, *[x.ptr for x in d], float(eps_psd), float(nu_max), on.ptr, oP.ptr,
              oc.ptr, ctx=ctx)
    nu, Psi, c = _abi.download_many([on, oP, oc])
    return replace(mn_state, nu=nu, Psi=Psi), c
