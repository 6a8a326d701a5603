"""SO(3)/SE(3) maps of fl_slam_poc/common/geometry/se3_jax.py on the GPU (gc_lie_batch).

Same names and argument conventions as the reference module; each function also accepts a
batch (leading dimensions) and evaluates every item in one launch. These run the exact device
routines the scan-path kernels use (gc_math.h), so a result here is what recompose, the world
pose, ξ_body, the Matrix-Fisher δ and the IMU/odom residuals compute on the device.
"""

from __future__ import annotations

import numpy as np

from .. import _abi

_OPS = {  # name: (op, in row, out row, out shape)
    "so3_exp": (0, 3, 9, (3, 3)),
    "so3_log": (1, 9, 3, (3,)),
    "se3_exp": (2, 6, 6, (6,)),
    "se3_log": (3, 6, 6, (6,)),
    "se3_V": (4, 3, 9, (3, 3)),
    "_se3_V_inv": (5, 3, 9, (3, 3)),
    "se3_compose": (6, 12, 6, (6,)),
    "se3_inverse": (7, 6, 6, (6,)),
}


def _run(name, x, ctx=None):
    op, n_in, n_out, oshape = _OPS[name]
    a = np.ascontiguousarray(x, dtype=np.float64)
    lead = a.shape[:-2] if name == "so3_log" else a.shape[:-1]
    if (name == "so3_log" and a.shape[-2:] != (3, 3)) or (name != "so3_log" and a.shape[-1] != n_in):
        raise ValueError(f"{name}: expected trailing shape {(3, 3) if name == 'so3_log' else (n_in,)}, got {a.shape}")
    n = int(np.prod(lead, dtype=np.int64))
    if n == 0:
        return np.zeros(lead + oshape)
    ctx = ctx or _abi.default_context()
    d_in = _abi.DeviceArray.from_host(ctx, a.reshape(n, n_in))
    d_out = _abi.DeviceArray(ctx, (n, n_out))
    _abi.call("gc_lie_batch", ctx.handle, op, n, d_in.ptr, d_out.ptr, ctx=ctx)
    return d_out.download().reshape(lead + oshape)


def so3_exp(omega, ctx=None):
    """se3_jax.py:259-301: rotation vector(s) (..., 3) -> R (..., 3, 3)."""
    return _run("so3_exp", omega, ctx)


def so3_log(R, ctx=None):
    """se3_jax.py:304-366: R (..., 3, 3) -> rotation vector(s) (..., 3)."""
    return _run("so3_log", R, ctx)


def se3_exp(xi, ctx=None):
    """se3_jax.py:473-504: twist [ρ, φ] (..., 6) -> pose [t, rotvec] (..., 6)."""
    return _run("se3_exp", xi, ctx)


def se3_log(T, ctx=None):
    """se3_jax.py:220-256: pose [t, rotvec] (..., 6) -> twist [ρ, φ] (..., 6)."""
    return _run("se3_log", T, ctx)


def se3_V(phi, ctx=None):
    """se3_jax.py:137-175."""
    return _run("se3_V", phi, ctx)


def _se3_V_inv(phi, ctx=None):
    """se3_jax.py:177-217."""
    return _run("_se3_V_inv", phi, ctx)


def se3_compose(a, b, ctx=None):
    """se3_jax.py:420-438: a ∘ b; a and b broadcast against each other."""
    a, b = np.broadcast_arrays(np.asarray(a, np.float64), np.asarray(b, np.float64))
    return _run("se3_compose", np.concatenate([a, b], axis=-1), ctx)


def se3_inverse(a, ctx=None):
    """se3_jax.py:441-453."""
    return _run("se3_inverse", a, ctx)


def se3_relative(a, b, ctx=None):
    """se3_jax.py:456-459: b⁻¹ ∘ a."""
    return se3_compose(se3_inverse(b, ctx), a, ctx)
