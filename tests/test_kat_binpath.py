"""Closed-form known answers for the bin path (a5-a8), run on the oracle and on the HIP path.

The reference holds no golden vectors for these operators, so besides the oracle
restatement they are pinned here by inputs whose answer follows from the reference formulas alone:

  * points exactly on the bin directions (binning.py:56-209): at τ = 0.1 the responsibilities are
    the rows of softmax(G/τ) with G the bins' Gram matrix and the bin index is the point's own bin;
    at τ = 0.003 the assignment is one-hot to 1e-14, so each bin's statistics are its own point's
    (N = w, s_dir = w d, S = w d dᵀ, p̄ = p w/(w + ε_mass), Σ_p the clamped rank-one lift residue, R̄ -> κ(1 - ε_R));
  * Matrix-Fisher with a scan that is the map rotated into the body frame by R_pred
    (matrix_fisher_evidence.py:155-256): H = R_pred M with M SPD, so R_mf = R_pred and δ = 0;
  * planar translation with scan centroids p̄_b = R̂ᵀ(c_b - t) (:413-499): every t_b = t, so
    t_wls = t up to the ε_mass lift.
"""

import numpy as np
import pytest

from oracle import gc_oracle as O

B = 48
ORIGIN = np.array([-0.065447, -0.100474, 0.108987])


def _points_on_bins():
    bins = O.fibonacci_atlas(B)
    r = 2.0 + 0.1 * np.arange(B)
    P = ORIGIN[None, :] + r[:, None] * bins
    w = np.linspace(0.5, 1.5, B)
    return bins, P, w


def _soft_reference(bins, tau):
    G = O.similarities(bins, bins)  # rows: points on bin k
    x = G / tau
    e = np.exp(x - x.max(1, keepdims=True))
    return e / e.sum(1, keepdims=True)


def _sigma_single(P, w, eps_mass=1e-12, eps_psd=1e-12):
    """Σ_p of a bin holding one point p of weight w (binning.py:175-190): Σ_raw = p pᵀ (c - c²) with
    c = w/(w + ε_mass) (the InvMass lift), rank one along p; PSD-clamped at ε_psd that is
    ε I + (|p|² (c - c²) - ε) p̂ p̂ᵀ."""
    c = w / (w + eps_mass)
    lam = np.einsum("bi,bi->b", P, P) * (c - c * c)
    ph = P / np.linalg.norm(P, axis=1, keepdims=True)
    return eps_psd * np.eye(3)[None] + (np.maximum(lam, eps_psd) - eps_psd)[:, None, None] * np.einsum(
        "bi,bj->bij", ph, ph)


def _rotation(seed):
    return O.so3_exp(np.random.default_rng(seed).normal(0, 0.6, 3))


def _mf_case(seed=3):
    rng = np.random.default_rng(seed)
    R = _rotation(seed)
    mN = rng.uniform(5, 50, B)
    m_dir = rng.normal(size=(B, 3))
    m_dir *= (mN * rng.uniform(0.3, 0.9, B) / np.linalg.norm(m_dir, axis=1))[:, None]
    A = rng.normal(size=(B, 3, 3)) * 0.3
    mS = (A @ np.swapaxes(A, 1, 2)) * mN[:, None, None]
    s_dir = m_dir @ R                       # body frame: Rᵀ m per bin
    sS = np.einsum("ji,bjk,kl->bil", R, mS, R)
    return R, s_dir, sS, mN.copy(), m_dir, mS, mN


def _planar_case(seed=4):
    rng = np.random.default_rng(seed)
    R_hat = _rotation(seed)
    t_true = np.array([1.3, -0.7, 0.25])
    c_map = rng.normal(0, 4, (B, 3))
    p_bar = (c_map - t_true[None, :]) @ R_hat     # R̂ᵀ (c - t)
    A = rng.normal(size=(B, 3, 3)) * 0.1
    Sig_p = A @ np.swapaxes(A, 1, 2) + 1e-3 * np.eye(3)
    Sig_c = Sig_p[::-1].copy()
    sN, Npos, mN = rng.uniform(1, 30, B), rng.uniform(1, 30, B), rng.uniform(1, 30, B)
    Bm = rng.normal(size=(B, 3, 3)) * 0.3
    mS = (Bm @ np.swapaxes(Bm, 1, 2)) * mN[:, None, None]
    return R_hat, t_true, p_bar, Sig_p, sN, c_map, Sig_c, Npos, mS, mN


# ----------------------------------------------------------------------------------- oracle
@pytest.mark.parametrize("tau", [0.1, 0.003])
def test_oracle_points_on_bins(tau):
    bins, P, w = _points_on_bins()
    d = O.point_directions(P, ORIGIN)
    sa = O.bin_soft_assign(d, bins, tau)
    np.testing.assert_array_equal(sa["bin_index"], np.arange(B))
    np.testing.assert_allclose(sa["resp"], _soft_reference(bins, tau), atol=1e-12, rtol=0)
    if tau == 0.003:
        np.testing.assert_allclose(sa["resp"], np.eye(B), atol=1e-14, rtol=0)
        mm = O.scan_bin_moment_match(P, None, w, sa["resp"], None, ORIGIN)
        np.testing.assert_allclose(mm["N"], w, rtol=1e-13)
        np.testing.assert_allclose(mm["s_dir"], w[:, None] * d, rtol=0, atol=1e-13)
        # p̄ = Σ w p / (N + ε_mass) (InvMass, primitives.py:195-212)
        np.testing.assert_allclose(mm["p_bar"], P * (w / (w + 1e-12))[:, None], rtol=0, atol=1e-13)
        np.testing.assert_allclose(mm["Sigma_p"], _sigma_single(P, w), rtol=0, atol=1e-13)
        np.testing.assert_allclose(mm["kappa"], O.kappa_scalar(1.0), rtol=1e-9)


def test_oracle_matrix_fisher_recovers_the_rotation():
    R, s_dir, sS, sN, m_dir, mS, mN = _mf_case()
    mf = O.matrix_fisher(R, s_dir, sS, sN, m_dir, mS, mN)
    np.testing.assert_allclose(mf["R_mf"], R, atol=1e-12, rtol=0)
    assert np.max(np.abs(mf["delta_rot"])) < 1e-12 and np.max(np.abs(mf["h_rot"])) < 1e-9


def test_oracle_planar_translation_recovers_the_offset():
    R_hat, t_true, p_bar, Sig_p, sN, c_map, Sig_c, Npos, mS, mN = _planar_case()
    tr = O.planar_translation(np.zeros(3), p_bar, Sig_p, sN, c_map, Sig_c, Npos, mS, mN, R_hat)
    np.testing.assert_allclose(tr["t_wls"], t_true, atol=1e-10, rtol=0)


# ----------------------------------------------------------------------------------- device
@pytest.mark.gpu
@pytest.mark.parametrize("tau", [0.1, 0.003])
def test_gpu_points_on_bins_contract_pair(ctx, tau):
    from gcslam.ops.binning import bin_soft_assign_batch, scan_bin_moment_match_batch, unpack_bin_stats
    bins, P, w = _points_on_bins()
    d = O.point_directions(P, ORIGIN)
    resp, idx, _ = bin_soft_assign_batch(d[None], bins, tau, ctx=ctx)
    np.testing.assert_array_equal(idx[0], np.arange(B))
    np.testing.assert_allclose(resp[0], _soft_reference(bins, tau), atol=1e-12, rtol=0)
    if tau == 0.003:
        st, _ = scan_bin_moment_match_batch(P[None], None, w[None], resp, None, ORIGIN, ctx=ctx)
        u = unpack_bin_stats(st[0])
        np.testing.assert_allclose(u["N"], w, rtol=1e-13)
        np.testing.assert_allclose(u["s_dir"], w[:, None] * d, rtol=0, atol=1e-13)
        np.testing.assert_allclose(u["p_bar"], P * (w / (w + 1e-12))[:, None], rtol=0, atol=1e-13)
        np.testing.assert_allclose(u["Sigma_p"], _sigma_single(P, w), rtol=0, atol=1e-13)
        np.testing.assert_allclose(u["kappa"], O.kappa_scalar(1.0), rtol=1e-9)


@pytest.mark.gpu
def test_gpu_points_on_bins_fused(ctx):
    """The fused a1->a6 kernel (no deskew: ξ = 0) at τ = 0.003: one-hot bins, p̄ = p, unit mean
    directions; N_b is the point's window-weighted mass (deskew_constant_twist.py:61-68)."""
    from gcslam import _abi
    from gcslam.ops.binning import unpack_bin_stats
    bins, P, w = _points_on_bins()
    t = np.linspace(100.0, 100.1, B)
    dP, dT, dW = (_abi.DeviceArray.from_host(ctx, a) for a in (P, t, w))
    scal = _abi.DeviceArray(ctx, 8)
    _abi.call("gc_budget_stats", ctx.handle, dW.ptr, B, B, scal.ptr, ctx=ctx)
    dX, dB = _abi.DeviceArray.from_host(ctx, np.zeros((1, 6))), _abi.DeviceArray.from_host(ctx, bins)
    st, ce = _abi.DeviceArray(ctx, (1, B, 38)), _abi.DeviceArray(ctx, (1, 8))
    oa, op = _abi.f64p(ORIGIN)
    _abi.call("gc_scan_bins_fused", ctx.handle, 1, B, B, B, dP.ptr, dT.ptr, dW.ptr, scal.ptr, 100.0, 100.1, dX.ptr,
              dB.ptr, 0.003, op, 1e-12, 1e-12, st.ptr, ce.ptr, 0, ctx=ctx)
    u = unpack_bin_stats(st.download()[0])
    wd = O.deskew_constant_twist(P, t, w, 100.0, 100.1, np.zeros(6))[1]
    np.testing.assert_allclose(u["N"], wd, rtol=1e-13)
    np.testing.assert_allclose(u["p_bar"], P * (wd / (wd + 1e-12))[:, None], rtol=0, atol=1e-13)
    np.testing.assert_allclose(u["s_dir"] / u["N"][:, None], O.point_directions(P, ORIGIN), rtol=0, atol=1e-13)


@pytest.mark.gpu
def test_gpu_matrix_fisher_recovers_the_rotation(ctx):
    from gcslam.belief import BeliefGaussianInfo
    from gcslam.ops import matrix_fisher_rotation_evidence
    R, s_dir, sS, sN, m_dir, mS, mN = _mf_case()
    # belief_pred at X_anchor = (0, log R) with a zero increment: its world rotation is R
    b = BeliefGaussianInfo("GC-RIGHT-01", "a", np.concatenate([np.zeros(3), O.so3_log(R)]), 0.0, np.zeros(22),
                           np.eye(22), np.zeros(22))
    res, cert, _ = matrix_fisher_rotation_evidence(b, s_dir, sS, sN, m_dir, mS, mN, ctx=ctx)
    np.testing.assert_allclose(res.R_mf, R, atol=1e-12, rtol=0)
    assert np.max(np.abs(res.delta_rot)) < 1e-11 and np.max(np.abs(res.h_rot)) < 1e-8


@pytest.mark.gpu
def test_gpu_planar_translation_recovers_the_offset(ctx):
    from gcslam.belief import BeliefGaussianInfo
    from gcslam.ops import planar_translation_evidence
    R_hat, t_true, p_bar, Sig_p, sN, c_map, Sig_c, Npos, mS, mN = _planar_case()
    b = BeliefGaussianInfo("GC-RIGHT-01", "a", np.zeros(6), 0.0, np.zeros(22), np.eye(22), np.zeros(22))
    res, cert, _ = planar_translation_evidence(b, p_bar, Sig_p, sN, c_map, Sig_c, Npos, mS, mN, R_hat, ctx=ctx)
    np.testing.assert_allclose(res.t_wls, t_true, atol=1e-10, rtol=0)
