"""GPU parity of the per-point / per-bin kernels (a1, a4, a5, a6 and the fused a1->a6 kernel)
against the CPU oracle on the same seeded inputs. Tolerances are written per assertion:
integer outputs (selection indices, bin indices) must be bit-exact; f64 values agree to
near machine precision (sin/cos/exp/eigh differ by ulps between libm/LAPACK and ocml/Jacobi)."""

import numpy as np
import pytest

from oracle import gc_oracle as O

pytestmark = pytest.mark.gpu


def _unit(rng, n):
    d = rng.normal(size=(n, 3))
    return d / np.linalg.norm(d, axis=1, keepdims=True)


def _rel(a, b):
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)


@pytest.mark.parametrize("n_in,cap", [(10000, 4096), (4096, 4096), (1000, 1500), (65536, 65536)])
def test_point_budget_matches_oracle(ctx, n_in, cap):
    from gcslam.ops import point_budget_resample
    rng = np.random.default_rng(1)
    P = rng.normal(size=(n_in, 3)) * 5
    T = np.sort(rng.uniform(0, 0.1, n_in))
    W = rng.uniform(0.1, 1.0, n_in)
    ring = rng.integers(0, 16, n_in).astype(np.uint8)
    res, cert, eff = point_budget_resample(P, T, W, ring=ring, n_points_cap=cap, ctx=ctx)
    ref = O.point_budget_resample(P, T, W, ring, None, cap)
    ns = ref["n_output"]
    assert res.n_output == ns
    np.testing.assert_array_equal(res.indices[:ns], ref["indices"])          # bit-exact selection
    assert np.all(res.indices[ns:] == -1)
    np.testing.assert_array_equal(res.points, ref["points"])                 # gathered bits
    np.testing.assert_array_equal(res.ring, ref["ring"])
    np.testing.assert_allclose(res.weights, ref["weights"], rtol=1e-13, atol=0)
    assert abs(res.total_mass_in - ref["total_mass_in"]) <= 1e-12 * ref["total_mass_in"]
    assert abs(cert.support.ess_total - ref["ess"]) <= 1e-10 * ref["ess"]
    assert abs(cert.total_trigger_magnitude() - ref["trig"]) < 1e-20


def test_deskew_matches_oracle(ctx):
    from gcslam.ops.deskew_constant_twist import deskew_batch, deskew_constant_twist
    rng = np.random.default_rng(2)
    n = 3000
    P = rng.normal(size=(n, 3)) * 8
    T = 100.0 + np.sort(rng.uniform(-0.01, 0.11, n))
    W = rng.uniform(0.0, 1.0, n)
    xis = np.array([[0.1, -0.02, 0.01, 0.0, 0.0, 0.03], [0.0, 0.0, 0.0, 0.0, 0.0, 0.0],
                    [0.5, 0.3, -0.2, 0.4, -0.3, 0.9], [1e-9, 0, 0, 1e-9, 0, 0]])
    pts, w_out, sw = deskew_batch(P, T, W, 100.0, 100.1, xis, ctx=ctx)
    for h in range(xis.shape[0]):
        rp, rw, ret = O.deskew_constant_twist(P, T, W, 100.0, 100.1, xis[h])
        np.testing.assert_allclose(pts[h], rp, atol=1e-12, rtol=0)
        np.testing.assert_allclose(w_out[h], rw, rtol=1e-13, atol=1e-300)
        assert abs(sw[h] / (W.sum() + 1e-12) - ret) < 1e-13
    res, cert, _ = deskew_constant_twist(P, T, W, 100.0, 100.1, xis[0], 3.0, "GC-RIGHT-01", "a", ctx=ctx)
    assert cert.exact and cert.support.ess_total == 3.0


@pytest.mark.parametrize("B,n", [(48, 4096), (20, 1000), (64, 777), (7, 300), (48, 65536), (48, 1000), (32, 333), (16, 97)])
def test_soft_assign_matches_oracle(ctx, B, n):
    from gcslam.ops.binning import bin_soft_assign_batch
    rng = np.random.default_rng(3 + B)
    D = np.stack([_unit(rng, n), _unit(rng, n)])
    bins = O.fibonacci_atlas(B)
    resp, idx, cert = bin_soft_assign_batch(D, bins, 0.1, ctx=ctx)
    for h in range(2):
        ref = O.bin_soft_assign(D[h], bins, 0.1)
        np.testing.assert_array_equal(idx[h], ref["bin_index"])              # bit-exact bin index
        np.testing.assert_allclose(resp[h], ref["resp"], atol=1e-14, rtol=0)
        assert abs(cert[h, 0] - ref["avg_entropy"]) < 1e-9
        assert abs(cert[h, 1] - ref["max_resp"]) < 1e-14
    np.testing.assert_allclose(resp.sum(-1), 1.0, atol=1e-12)                # rows sum to 1


@pytest.mark.parametrize("tau,norm", [(0.01, 1.0), (1.0, 1.0), (0.1, 3.7), (0.1, 0.05), (1e-4, 1.0), (0.01, 40.0)])
def test_soft_assign_row_max_shift_any_tau_and_norm(ctx, tau, norm):
    """jax.nn.softmax shifts by the row maximum (binning.py:68-69), so the drop-in must accept any
    τ > 0 and non-unit directions (at τ = 1e-4 the bound shift (S - 1)/τ would underflow every
    exp). Tolerance: x = (S - S_max)/τ rounds at ulp(|S|/τ), so |ΔR| <= ~4 ulp(|S|/τ)."""
    from gcslam.ops.binning import bin_soft_assign_batch
    rng = np.random.default_rng(11)
    n = 3000
    D = (_unit(rng, n) * norm * rng.uniform(0.5, 1.5, (n, 1)))[None]
    bins = O.fibonacci_atlas(48)
    resp, idx, cert = bin_soft_assign_batch(D, bins, tau, ctx=ctx)
    ref = O.bin_soft_assign(D[0], bins, tau)
    tol = 4 * np.spacing(1.5 * norm / tau) + 1e-15
    np.testing.assert_array_equal(idx[0], ref["bin_index"])
    np.testing.assert_allclose(resp[0], ref["resp"], atol=tol, rtol=0)
    assert np.all(np.isfinite(resp)) and np.all(resp >= 0.0)
    np.testing.assert_allclose(resp.sum(-1), 1.0, atol=1e-12)
    assert abs(cert[0, 0] - ref["avg_entropy"]) < 1e-9 + 48 * tol
    assert abs(cert[0, 1] - ref["max_resp"]) < 1e-14 + tol


def test_fused_rejects_tau_below_table_floor(ctx):
    """The fused kernel's table exp covers arguments down to -2/τ for τ >= GC_FUSED_TAU_MIN; below
    it the call fails loudly (ValueError) instead of wrapping the exponent."""
    from gcslam import _abi
    H, n = 1, 512
    d = _abi.DeviceArray(ctx, (n, 3)); d.zero()
    t = _abi.DeviceArray(ctx, n); t.zero()
    scal = _abi.DeviceArray(ctx, 8); scal.zero()
    xi, bins = _abi.DeviceArray(ctx, (H, 6)), _abi.DeviceArray.from_host(ctx, O.fibonacci_atlas(48))
    st, ce = _abi.DeviceArray(ctx, (H, 48, 38)), _abi.DeviceArray(ctx, (H, 8))
    oa, op = _abi.f64p([0.0, 0.0, 0.0])
    with pytest.raises(ValueError, match="tau"):
        _abi.call("gc_scan_bins_fused", ctx.handle, H, n, n, 48, d.ptr, t.ptr, t.ptr, scal.ptr, 0.0, 0.1, xi.ptr,
                  bins.ptr, 1e-3, op, 1e-12, 1e-12, st.ptr, ce.ptr, 0, ctx=ctx)


def test_bin_index_ties_resolve_to_lowest_index(ctx):
    from gcslam.ops.binning import bin_soft_assign_batch
    bins = np.array([[1.0, 0, 0], [0, 1.0, 0], [1.0, 0, 0], [0, 0, 1.0]])
    D = np.array([[[1.0, 0, 0], [0, 0, 1.0], [0.6, 0.8, 0.0]]])
    _, idx, _ = bin_soft_assign_batch(D, bins, 0.1, ctx=ctx)
    np.testing.assert_array_equal(idx[0], [0, 3, 1])


def _check_stats(stats, cert, ref, rtol=1e-10):
    from gcslam.ops.binning import unpack_bin_stats
    u = unpack_bin_stats(stats)
    scale = max(np.max(np.abs(ref["N"])), 1e-300)
    np.testing.assert_allclose(u["N"], ref["N"], atol=rtol * scale, rtol=0)
    np.testing.assert_allclose(u["s_dir"], ref["s_dir"], atol=rtol * scale, rtol=0)
    np.testing.assert_allclose(u["S_dir_scatter"], ref["S_dir_scatter"], atol=rtol * scale, rtol=0)
    np.testing.assert_allclose(u["p_bar"], ref["p_bar"], atol=1e-9, rtol=0)
    np.testing.assert_allclose(u["Sigma_p"], ref["Sigma_p"], atol=1e-8, rtol=0)
    np.testing.assert_allclose(u["kappa"], ref["kappa"], rtol=1e-8, atol=1e-10)
    assert abs(cert[0] - ref["ess"]) <= 1e-9 * ref["ess"]
    assert abs(cert[1] - ref["support_frac"]) < 1e-12
    assert abs(cert[2] - ref["psd_delta"]) < 1e-8
    assert abs(cert[3] - ref["max_eps_ratio"]) <= 1e-9 * ref["max_eps_ratio"] + 1e-300


@pytest.mark.parametrize("B,n,with_cov", [(48, 4096, False), (48, 2500, True), (20, 1000, False),
                                          (64, 600, True)])
def test_moment_match_matches_oracle(ctx, B, n, with_cov):
    from gcslam.ops.binning import scan_bin_moment_match_batch
    rng = np.random.default_rng(5)
    H = 2
    P = rng.normal(size=(H, n, 3)) * 6
    W = rng.uniform(0.0, 1.0, (H, n))
    lam = rng.uniform(0.5, 1.5, (H, n))
    covs = None
    if with_cov:
        A = rng.normal(size=(H, n, 3, 3)) * 0.01
        covs = A @ np.swapaxes(A, -1, -2)
    o = np.array([-0.065447, -0.100474, 0.108987])
    bins = O.fibonacci_atlas(B)
    R = np.stack([O.bin_soft_assign(O.point_directions(P[h], o), bins)["resp"] for h in range(H)])
    stats, cert = scan_bin_moment_match_batch(P, covs, W, R, lam, o, ctx=ctx)
    for h in range(H):
        ref = O.scan_bin_moment_match(P[h], None if covs is None else covs[h], W[h], R[h], lam[h], o)
        _check_stats(stats[h], cert[h], ref)


@pytest.mark.parametrize("n_in,cap,B,iters,tau", [
    (4096, 4096, 48, 0, 0.1), (5000, 2048, 48, 0, 0.1), (3000, 3500, 48, 0, 0.1), (2000, 2000, 20, 0, 0.1),
    # the iteration counts the benchmark runs (16 at 64k x 256, 8 for a 32-hypothesis shard) and
    # caps that leave a partial last chunk (the PAD specialisation at several iterations)
    (65536, 65536, 48, 16, 0.1), (65536, 65536, 48, 8, 0.1), (5000, 5000, 48, 2, 0.1),
    (20000, 20000, 48, 8, 0.1), (65536, 30000, 48, 16, 0.1), (3000, 3000, 20, 4, 0.1),
    # C2 at full size with the automatic geometry (H = 3 -> one iteration per workgroup)
    (65536, 65536, 48, 0, 0.1),
    # other temperatures (down to the fused kernel's floor)
    (4096, 4096, 48, 4, 0.01), (4096, 4096, 48, 2, 1.0), (4096, 4096, 48, 0, 0.003)])
def test_fused_bins_match_contract_chain(ctx, n_in, cap, B, iters, tau):
    """Fused a1->a4->a5->a6 == oracle chain budget -> deskew -> dirs -> soft assign -> moments."""
    _fused_vs_chain(ctx, n_in, cap, B, iters, tau, np.array([[0.02, 0.0, 0.0, 0.0, 0.0, 0.03],
                                                             [0.0, 0.01, 0.0, 0.01, -0.01, -0.02], [0.0] * 6]))


@pytest.mark.parametrize("n_in,iters", [(4096, 0), (8192, 2), (5000, 2)])
def test_fused_bins_fast_rotation_match_contract_chain(ctx, n_in, iters):
    """The fused kernel's other two deskew forms: rotations past the short series (θ² > 0.04 over
    the scan: the nine-term series) and past θ² = 1 (the closed form with sin / cos), in waves that
    mix them with the short form (θ = α|ω| grows with the point's time)."""
    xis = np.array([[0.3, -0.1, 0.05, 0.3, -0.2, 0.4],      # |ω| 0.54: short, then the series
                    [0.1, 0.0, 0.2, 1.2, 0.5, -0.9],        # |ω| 1.58: all three forms
                    [-0.5, 0.4, 0.0, -2.5, 1.0, 2.0]])      # |ω| 3.35: mostly the closed form
    _fused_vs_chain(ctx, n_in, n_in, 48, iters, 0.1, xis)


def _fused_vs_chain(ctx, n_in, cap, B, iters, tau, xis):
    from gcslam import _abi
    from gcslam.synth import make_scan
    s = make_scan(0, n_az=max(1, n_in // 16))
    P, T, W = s["points"][:n_in], s["timestamps"][:n_in], s["weights"][:n_in]
    n_in = P.shape[0]
    o = np.array([-0.065447, -0.100474, 0.108987])
    bins = O.fibonacci_atlas(B)
    H = xis.shape[0]
    dP, dT, dW = (_abi.DeviceArray.from_host(ctx, a) for a in (P, T, W))
    scal = _abi.DeviceArray(ctx, 8)
    _abi.call("gc_budget_stats", ctx.handle, dW.ptr, n_in, cap, scal.ptr, ctx=ctx)
    dX, dB = _abi.DeviceArray.from_host(ctx, xis), _abi.DeviceArray.from_host(ctx, bins)
    st = _abi.DeviceArray(ctx, (H, B, 38)); ce = _abi.DeviceArray(ctx, (H, 8))
    oa, op = _abi.f64p(o)
    _abi.call("gc_scan_bins_fused", ctx.handle, H, n_in, cap, B, dP.ptr, dT.ptr, dW.ptr, scal.ptr,
              s["scan_start"], s["scan_end"], dX.ptr, dB.ptr, tau, op, 1e-12, 1e-12, st.ptr, ce.ptr, iters,
              ctx=ctx)
    stats, cert = st.download(), ce.download()
    bud = O.point_budget_resample(P, T, W, None, None, cap)
    for h in range(H):
        p0, wd, ret = O.deskew_constant_twist(bud["points"], bud["timestamps"], bud["weights"],
                                              s["scan_start"], s["scan_end"], xis[h])
        sa = O.bin_soft_assign(O.point_directions(p0, o), bins, tau)
        ref = O.scan_bin_moment_match(p0, None, wd, sa["resp"], None, o)
        _check_stats(stats[h], cert[h], ref, rtol=1e-10)
        # the logits round at ulp(1/τ): entropy within ~B·ulp(1/τ), max responsibility within
        # a few ulp(1/τ)
        assert abs(cert[h, 4] - sa["avg_entropy"]) < 1e-9 + 48 * np.spacing(1.0 / tau)
        assert abs(cert[h, 5] - sa["max_resp"]) < 1e-12 + 4 * np.spacing(1.0 / tau)
        assert abs(cert[h, 6] / (bud["weights"].sum() + 1e-12) - ret) < 1e-12


def test_fused_is_bit_reproducible(ctx):
    """Full-size properties at the benchmark geometry (C3: 65,536 points x 256 hypotheses, 16
    iterations per workgroup): two runs agree bit for bit and Σ_b N_b = Σ_n w_deskew for every
    hypothesis (softmax rows sum to one)."""
    from gcslam import _abi
    from gcslam.synth import make_scan
    s = make_scan(1, n_az=4096)
    n = s["points"].shape[0]
    bins = O.fibonacci_atlas(48)
    H = 256
    xis = np.random.default_rng(9).normal(size=(H, 6)) * 0.02
    dP, dT, dW = (_abi.DeviceArray.from_host(ctx, s[k]) for k in ("points", "timestamps", "weights"))
    scal = _abi.DeviceArray(ctx, 8)
    _abi.call("gc_budget_stats", ctx.handle, dW.ptr, n, n, scal.ptr, ctx=ctx)
    dX, dB = _abi.DeviceArray.from_host(ctx, xis), _abi.DeviceArray.from_host(ctx, bins)
    outs = []
    for _ in range(2):
        st = _abi.DeviceArray(ctx, (H, 48, 38)); ce = _abi.DeviceArray(ctx, (H, 8))
        oa, op = _abi.f64p([-0.065447, -0.100474, 0.108987])
        _abi.call("gc_scan_bins_fused", ctx.handle, H, n, n, 48, dP.ptr, dT.ptr, dW.ptr, scal.ptr,
                  s["scan_start"], s["scan_end"], dX.ptr, dB.ptr, 0.1, op, 1e-12, 1e-12, st.ptr, ce.ptr, 0, ctx=ctx)
        outs.append((st.download(), ce.download()))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    # mass conservation: Σ_b N_b = Σ_n w_deskew (softmax rows sum to one)
    np.testing.assert_allclose(outs[0][0][:, :, 0].sum(1), outs[0][1][:, 6], rtol=1e-12)


@pytest.mark.parametrize("d", [22, 6, 3, 2, 1, 5, 7, 23, 40, 64, 100])
def test_psd_projection_matches_oracle(ctx, d):
    """domain_projection_psd_core takes any square matrix (primitives.py:80-123): even d <= 22 on
    the fixed-size path, odd / larger d padded (LDS up to 64, global workspace beyond).
    Tolerance 1e-12 x scale x max(1, d/16) (Jacobi vs LAPACK eigh rounding grows with d)."""
    from gcslam.ops.primitives import domain_projection_psd_batch
    rng = np.random.default_rng(7 + d)
    A = rng.normal(size=(5, d, d))
    M = A @ np.swapaxes(A, 1, 2) - 0.5 * np.eye(d)[None]  # some negative eigenvalues
    M[0] = np.eye(d)
    M[1] = np.zeros((d, d))
    M[2, 0, -1] += 0.3  # asymmetric
    Mp, c = domain_projection_psd_batch(M, 1e-12, ctx=ctx)
    for i in range(5):
        rp, rc = O.psd_project(M[i])
        sc = max(np.max(np.abs(M[i])), 1.0) * max(1.0, d / 16)
        np.testing.assert_allclose(Mp[i], rp, atol=1e-12 * sc, rtol=0)
        np.testing.assert_allclose(c[i, [1, 5]], rc[[1, 5]], atol=1e-12 * sc)
        np.testing.assert_allclose(c[i, 2:4], rc[2:4], atol=1e-12 * sc)
        assert abs(c[i, 0] - rc[0]) < 1e-10 * sc


def test_kappa_matches_oracle(ctx):
    from gcslam.ops import kappa_from_resultant_batch
    R = np.concatenate([np.linspace(-0.1, 1.1, 1001), [0.1, 0.3, 0.5, 0.7, 0.85, 1 - 1e-6]])
    # rtol 1e-10: the reference's own batch-vs-scalar tolerance (test_audit_invariants.py:412-426)
    np.testing.assert_allclose(kappa_from_resultant_batch(R, ctx=ctx), O.kappa_batch(R), rtol=1e-10, atol=1e-12)
