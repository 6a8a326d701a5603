"""BinSoftAssign / ScanBinMomentMatch (archive/legacy_operators/binning.py:34-324) and the
Fibonacci bin atlas (archive/bin_atlas.py:30-75) on the GPU."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import numpy as np

from .. import _abi
from ..certificates import CertBundle, ExpectedEffect, InfluenceCert, SupportCert
from ..constants import GC_B_BINS, GC_CHART_ID, GC_EPS_MASS, GC_EPS_PSD, GC_TAU_SOFT_ASSIGN


@dataclass
class BinAtlas:
    dirs: np.ndarray  # (B, 3)


def create_fibonacci_atlas(n_bins: int = GC_B_BINS) -> BinAtlas:
    """Init-time Fibonacci lattice (bin_atlas.py:40-75; the reference builds it un-jitted)."""
    i = np.arange(n_bins, dtype=np.float64) + 0.5
    phi = np.arccos(1 - 2 * i / n_bins)
    theta = np.pi * (1 + np.sqrt(5)) * i
    d = np.stack([np.sin(phi) * np.cos(theta), np.sin(phi) * np.sin(theta), np.cos(phi)], axis=1)
    return BinAtlas(dirs=d / (np.linalg.norm(d, axis=1, keepdims=True) + GC_EPS_MASS))


@dataclass
class BinSoftAssignResult:
    responsibilities: np.ndarray  # (N, B)
    bin_index: np.ndarray = None  # (N,) int32 argmax of the similarities (integer contract)


@dataclass
class ScanBinStats:
    N: np.ndarray
    s_dir: np.ndarray
    S_dir_scatter: np.ndarray
    p_bar: np.ndarray
    Sigma_p: np.ndarray
    kappa_scan: np.ndarray


def unpack_bin_stats(rec: np.ndarray):
    """(..., B, GC_BIN_STATS) record -> dict of named arrays (include/gcslam.h layout)."""
    sh = rec.shape[:-1]
    return dict(N=rec[..., 0], s_dir=rec[..., 1:4], S_dir_scatter=rec[..., 4:13].reshape(sh + (3, 3)),
                p_bar=rec[..., 13:16], Sigma_p=rec[..., 16:25].reshape(sh + (3, 3)), kappa=rec[..., 25],
                sum_p=rec[..., 26:29], sum_ppT=rec[..., 29:38].reshape(sh + (3, 3)))


def _shape(x):
    return x.shape if isinstance(x, _abi.DeviceArray) else np.shape(x)


def point_directions(points, direction_origin, eps_mass: float = GC_EPS_MASS, ctx=None, device_out: bool = False):
    """dirs = (p − o) / (‖p − o‖ + eps) (pipeline.py:589-593), host or DeviceArray points (N, 3)."""
    ctx = ctx or _abi.default_context()
    sh = _shape(points)
    n = int(np.prod(sh)) // 3
    dp = _abi.device_input(ctx, points, np.float64, (n, 3))
    oa, op = _abi.f64p(np.asarray(direction_origin, np.float64).reshape(3))
    out = _abi.DeviceArray(ctx, (n, 3))
    _abi.call("gc_point_directions", ctx.handle, n, dp.ptr, op, float(eps_mass), out.ptr, ctx=ctx)
    return out if device_out else out.download()


def bin_soft_assign_batch(dirs, bins, tau=GC_TAU_SOFT_ASSIGN, ctx=None, device_out: bool = False):
    """(H, N, 3) directions (host or DeviceArray) -> resp (H, N, B), bin_index (H, N), cert (H, 2)."""
    ctx = ctx or _abi.default_context()
    sh = _shape(dirs)
    H, n = (1, sh[0]) if len(sh) == 2 else (sh[0], sh[1])
    Bd = np.ascontiguousarray(bins, dtype=np.float64).reshape(-1, 3)
    B = Bd.shape[0]
    if not 1 <= B <= 64:
        raise ValueError(f"bin count must be in [1, 64], got {B}")
    dd, db = _abi.upload_many(ctx, (dirs, Bd))
    dd = _abi.device_input(ctx, dd, np.float64, (H, n, 3))
    dr, di, dc = _abi.alloc_many(ctx, [(H, n, B), ((H, n), np.int32), (H, 2)])
    _abi.call("gc_bin_soft_assign", ctx.handle, H, n, B, dd.ptr, db.ptr, float(tau), dr.ptr, di.ptr, dc.ptr,
              ctx=ctx)
    if device_out:
        return dr, di, dc.download()
    return tuple(_abi.download_many([dr, di, dc]))


def bin_soft_assign(point_directions, bin_directions, tau: float = GC_TAU_SOFT_ASSIGN,
                    chart_id: str = GC_CHART_ID, anchor_id: str = "initial", ctx=None, device_out: bool = False
                    ) -> Tuple[BinSoftAssignResult, CertBundle, ExpectedEffect]:
    """Host or DeviceArray directions (N, 3); with device_out the N x B responsibilities (and bin
    indices) stay in HBM for scan_bin_moment_match."""
    sh = _shape(point_directions)
    if len(sh) != 2 or sh[1] != 3:
        raise ValueError(f"point_directions must be (N, 3), got {sh}")
    resp, idx, c = bin_soft_assign_batch(point_directions, bin_directions, tau, ctx, device_out)
    avg_entropy, max_resp = float(c[0, 0]), float(c[0, 1])
    cert = CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id,
                                   support=SupportCert(ess_total=float(np.exp(avg_entropy)),
                                                       support_frac=max_resp))
    if device_out:
        n, B = resp.shape[1], resp.shape[2]
        r = BinSoftAssignResult(responsibilities=resp.view((n, B)), bin_index=idx.view((n,)))
    else:
        r = BinSoftAssignResult(responsibilities=resp[0], bin_index=idx[0])
    return r, cert, ExpectedEffect(objective_name="predicted_assignment_entropy", predicted=avg_entropy)


def scan_bin_moment_match_batch(points, point_covariances, weights, responsibilities, point_lambda=None,
                                direction_origin=None, eps_psd=GC_EPS_PSD, eps_mass=GC_EPS_MASS, ctx=None):
    """Batched contract kernel: (H,N,3) points etc. -> (stats (H,B,38), cert (H,8))."""
    ctx = ctx or _abi.default_context()
    sh = _shape(points)
    H, n = (1, sh[0]) if len(sh) == 2 else (sh[0], sh[1])
    rsh = _shape(responsibilities)
    B = int(np.prod(rsh)) // (H * n)
    o = np.zeros(3) if direction_origin is None else np.asarray(direction_origin, np.float64).reshape(-1)
    if o.shape[0] != 3:
        raise ValueError(f"direction_origin must be (3,), got {o.shape}")
    dev = [_abi.device_input(ctx, points, np.float64, (H, n, 3)),
           None if point_covariances is None else _abi.device_input(ctx, point_covariances, np.float64, (H, n, 9)),
           _abi.device_input(ctx, weights, np.float64, (H, n)),
           _abi.device_input(ctx, responsibilities, np.float64, (H, n, B)),
           None if point_lambda is None else _abi.device_input(ctx, point_lambda, np.float64, (H, n))]
    ptr = [d.ptr if d is not None else None for d in dev]
    ds, dc = _abi.alloc_many(ctx, [(H, B, _abi.GC_BIN_STATS), (H, _abi.GC_BIN_CERT)])
    oa, op = _abi.f64p(o)
    _abi.call("gc_scan_bin_moment_match", ctx.handle, H, n, B, ptr[0], ptr[1], ptr[2], ptr[3], ptr[4], op,
              float(eps_psd), float(eps_mass), ds.ptr, dc.ptr, ctx=ctx)
    return tuple(_abi.download_many([ds, dc]))


def scan_bin_moment_match(points, point_covariances, weights, responsibilities, point_lambda=None,
                          direction_origin=None, eps_psd: float = GC_EPS_PSD, eps_mass: float = GC_EPS_MASS,
                          chart_id: str = GC_CHART_ID, anchor_id: str = "initial", ctx=None
                          ) -> Tuple[ScanBinStats, CertBundle, ExpectedEffect]:
    n = _shape(points)[0]
    if point_lambda is not None and int(np.prod(_shape(point_lambda))) != n:
        raise ValueError(f"point_lambda must be (N,), got {_shape(point_lambda)} for N={n}")
    covs = None
    if point_covariances is not None:
        covs = point_covariances
        if not isinstance(covs, _abi.DeviceArray):
            covs = np.asarray(covs, dtype=np.float64)
            if not np.any(covs):
                covs = None  # all-zero covariances add nothing: skip the 9 extra streams
    stats, c = scan_bin_moment_match_batch(points, covs, weights, responsibilities, point_lambda, direction_origin,
                                           eps_psd, eps_mass, ctx)
    u = unpack_bin_stats(stats[0])
    res = ScanBinStats(N=u["N"], s_dir=u["s_dir"], S_dir_scatter=u["S_dir_scatter"], p_bar=u["p_bar"],
                       Sigma_p=u["Sigma_p"], kappa_scan=u["kappa"])
    c = c[0]
    cert = CertBundle.create_approx(
        chart_id=chart_id, anchor_id=anchor_id, triggers=["ScanBinMomentMatch"],
        support=SupportCert(ess_total=float(c[0]), support_frac=float(c[1])),
        influence=InfluenceCert(psd_projection_delta=float(c[2]), mass_epsilon_ratio=float(c[3])))
    return res, cert, ExpectedEffect(objective_name="predicted_ess", predicted=float(c[0]))
