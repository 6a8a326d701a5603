"""Parity at the geometries BASELINE.json names, through the shipped batched pipeline (C-ABI
gc_pipeline_*), against the oracle's restatement of the reference pipeline.

  C2  65,536 points, H = 1: the whole scan (fused kernel at its automatic geometry).
  C3  65,536 points x 256 hypotheses, IMU/odom branch computed: exactly the bench.py workload,
      fused kernel at 16 iterations per workgroup, the H = 256 combine layout.
  C5  131,072 points (budget stride 2 -> 65,536) x 1024 hypotheses.

The oracle costs ~0.3 s per hypothesis at 64k points, so C3/C5 compare sampled hypotheses
(first, second, middle, last) per scan; everything that couples hypotheses (IW accumulation,
barycenter combine, map update) is checked by feeding the GPU's own per-hypothesis outputs of ALL
hypotheses into the oracle's combine / IW apply / map update. Each scan re-seeds the oracle from
the GPU's state before the scan (beliefs, IW, map), so the comparison measures one scan's error
and does not accumulate drift.

Tolerances (per assertion): world pose 1e-6 abs (north star); covariance: the pose block of
Σ = (L + ε_lift I)⁻¹ 1e-6 abs (north star), the full Σ relative to its largest entry 1e-8 (the
unobserved directions keep the 1e-6 prior precision, so Σ reaches ~1e6 there and an absolute
1e-6 would demand 1e-12 relative rounding, below what two different f64 factorisation orders
agree to); information matrices 1e-8 relative; bin statistics 1e-10 relative.
"""

import numpy as np
import pytest

from oracle import gc_oracle as O
from oracle import cases

pytestmark = pytest.mark.gpu

EPS_LIFT = 1e-9


_FAILS = []


def _close(a, b, rel, abs_=0.0, what=""):
    """Records a failure (all of a test's comparisons are reported together at its end)."""
    a, b = np.asarray(a), np.asarray(b)
    err = np.max(np.abs(a - b))
    scale = max(np.max(np.abs(b)), 1e-300)
    if not err <= rel * scale + abs_:
        _FAILS.append(f"{what}: max|diff| {err:.3e} vs scale {scale:.3e} (bound {rel:.0e} rel + {abs_:.0e} abs)")


@pytest.fixture(autouse=True)
def _report():
    _FAILS.clear()
    yield
    assert not _FAILS, "\n".join(_FAILS[:60])


def _cert6(dev, ref, what):
    """The reference's cert_vec [projection_delta, sym_delta, eig_min, eig_max, cond, nnc]
    (primitives.py:80-123) of one projection: both deltas within the rounding of the two
    V diag(λ) Vᵀ reconstructions (~1e-16 of the spectrum's scale per entry), the clamped eigenvalue
    extremes at the absolute accuracy of eigh (~1e-12 of the largest), cond = eig_max / eig_min of the
    device's own extremes and within 1e-6 of the reference's where eig_min is resolved to that
    relative accuracy, near-null count exact."""
    dev, ref = np.asarray(dev), np.asarray(ref)
    sc = max(abs(ref[3]), 1e-300)
    _close(dev[0:2], ref[0:2], 0.0, 1e-12 * sc, f"{what} deltas")
    _close(dev[3], ref[3], 1e-10, 0.0, f"{what} eig_max")
    _close(dev[2], ref[2], 0.0, 1e-12 * sc, f"{what} eig_min")
    _close(dev[4], dev[3] / dev[2], 1e-15, 0.0, f"{what} cond (own extremes)")
    if ref[2] > 1e-5 * ref[3]:
        _close(dev[4], ref[4], 1e-6, 0.0, f"{what} cond")
    _close(dev[5], ref[5], 0.0, 0.0, f"{what} near-null count")


def _cov(L):
    return np.linalg.inv(L + EPS_LIFT * np.eye(L.shape[-1]))


def _record_to_map(rec):
    B = rec.shape[0]
    return O.MapStats(rec[:, 0:3].copy(), rec[:, 3:12].reshape(B, 3, 3).copy(), rec[:, 12].copy(),
                      rec[:, 13].copy(), rec[:, 14:17].copy(), rec[:, 17:26].reshape(B, 3, 3).copy())


def _pipeline(case, ctx, H, cap, io_computed, rank=0, world=1, geometry_hyps=0):
    from gcslam.pipeline import BatchedScanPipeline, PipelineConfig
    n_in = case["scans"][0]["points"].shape[0]
    pipe = BatchedScanPipeline(H, n_in, PipelineConfig(n_points_cap=cap), rank=rank, world_size=world, ctx=ctx,
                               geometry_hyps=geometry_hyps)
    hy = case["hyp"]
    sl = slice(pipe.h0, pipe.h1)
    pipe.set_beliefs(hy["X_anchor"][sl], hy["z_lin"][sl], hy["L"][sl], hy["h"][sl], hy["stamp"][sl])
    pipe.set_weights(hy["weights"])
    if io_computed:
        pipe.set_io_mode(True)
    else:
        pipe.set_io_evidence(*(a[sl] for a in case["io"]))
    pipe.set_iw(*case["iw"])
    pipe.set_map(case["map_record"])
    return pipe


def _run_and_compare(ctx, case, H, cap, sample, n_scans, io_computed, pipe=None, hooks=None):
    """pipe: a BatchedScanPipeline, or any object with its scan / getter surface (the sharded
    view of test_gpu_shards.py); default: one unsharded pipeline. hooks: (before(k), after(k, x))
    run around each scan (x = before's return), e.g. the attached PrimitiveMap's own check."""
    cfg = O.PipeConfig(n_points_cap=cap)
    bins = case["bins"]
    pipe = pipe if pipe is not None else _pipeline(case, ctx, H, cap, io_computed)
    weights = case["hyp"]["weights"]
    floor = 0.01 / H
    for k, s in enumerate(case["scans"][:n_scans]):
        # the oracle's inputs: the GPU's state before this scan
        bel0, iw0, mp0 = pipe.get_beliefs(), pipe.get_iw(), pipe.get_map()
        mapst = _record_to_map(mp0["map"])
        Q = O.iw_process_Q(iw0["nu_proc"], iw0["Psi_proc"])
        Sga = (O.iw_meas_mode(iw0["nu_meas"], iw0["Psi_meas"], 0), O.iw_meas_mode(iw0["nu_meas"], iw0["Psi_meas"], 1))
        md = O.map_derived(mapst)
        scan = cases.scan_input(s)
        hx = hooks[0](k) if hooks else None
        pipe.stage_scan(0, s)
        pipe.run_scan(0, s, k)
        ctx.sync()
        if hooks:
            hooks[1](k, hx)
        diag = pipe.hyp_diag()
        hcond = pipe.hyp_conditioning()
        stats, bcert, xi = pipe.bin_stats()
        bel = pipe.get_beliefs()
        dPp, dPm, Sig = pipe.hyp_stats()
        pcert = pipe.projection_certs()
        res0 = None
        for i in sample:
            b_prev = O.Belief(bel0["X_anchor"][i].copy(), bel0["z_lin"][i].copy(), bel0["L"][i].copy(),
                              bel0["h"][i].copy(), float(bel0["stamp"][i]))
            io = None if io_computed else O.IOEvidence(case["io"][0][i], case["io"][1][i], case["io"][2][i, 0:3],
                                                       case["io"][2][i, 3:6], *case["io"][2][i, 6:10])
            # an inactive clamp's projection delta taken as its exact-arithmetic 0 (the device's value,
            # certified by Cholesky / Sturm counts) instead of the reference's ~1e-16 ||M|| rounding of
            # V diag(λ) Vᵀ, so T compares tightly; the reference-rounding T is pinned against the
            # tests/golden c3_all / c5_all fixtures at 1e-7 relative (test_c3_every_hypothesis_...)
            with O.exact_inactive_deltas():
                r = O.scan_hypothesis(b_prev, scan, Q, io, mapst, md, bins, cfg, Sga)
            if i == 0:
                res0 = r
            tag = f"scan{k} hyp{i}"
            _close(xi[i], r["xi_body"], 1e-9, 1e-12, f"{tag} xi_body")
            _close(stats[i, :, 0], r["moments"]["N"], 1e-10, 0, f"{tag} bin N")
            _close(stats[i, :, 1:4], r["moments"]["s_dir"], 1e-10, 0, f"{tag} bin s_dir")
            _close(stats[i, :, 13:16], r["moments"]["p_bar"], 1e-10, 1e-12, f"{tag} bin p_bar")
            _close(stats[i, :, 16:25].reshape(-1, 3, 3), r["moments"]["Sigma_p"], 1e-7, 1e-12, f"{tag} Sigma_p")
            _close(bcert[i, 4], r["assign"]["avg_entropy"], 1e-9, 0, f"{tag} avg entropy")
            _close(diag[i, 24:27], O.so3_log(r["mf"]["R_mf"]), 1e-7, 1e-10, f"{tag} R_mf")
            _close(diag[i, 21:24], r["planar"]["t_wls"], 1e-7, 1e-10, f"{tag} t_wls")
            # certificate magnitudes with exact inactive deltas on both sides (above): T, the sum over
            # every certificate, to 1e-10 relative (against the reference's rounding it differs by
            # ~2e-8 relative: ||L_post|| reaches ~1e8 at 64k points)
            _close(diag[i, 6], r["T"], 1e-10, 1e-12, f"{tag} T")
            _close(diag[i, 18], r["mf"]["trig"], 0, 1e-9, f"{tag} MF trigger")
            _close(diag[i, 19], r["planar"]["trig"], 0, 1e-9, f"{tag} planar trigger")
            _close(diag[i, 8], r["alpha"], 0, 1e-12, f"{tag} alpha")
            _close(diag[i, 9:11], [r["s_dt"], r["s_ex"]], 0, 1e-12, f"{tag} excitation scales")
            _close(diag[i, 13], r["cond6"], 1e-6, 0, f"{tag} cond_pose6")
            _close(bcert[i, 2], r["moments"]["psd_delta"], 0, 1e-10, f"{tag} moment psd delta")
            _close(bcert[i, 3], r["moments"]["max_eps_ratio"], 1e-8, 1e-300, f"{tag} moment mass-eps ratio")
            _close(bcert[i, 7], r["moments"]["trig"], 0, 1e-10, f"{tag} moment trigger")
            _close(diag[i, 7], r["beta"], 0, 1e-10, f"{tag} beta")
            b = r["belief"]
            _close(diag[i, 0:6], r["pose"], 0.0, 1e-6, f"{tag} world pose")             # north-star bar
            _close(bel["X_anchor"][i], b.X_anchor, 0.0, 1e-6, f"{tag} X_anchor")
            _close(bel["L"][i], b.L, 1e-8, 0.0, f"{tag} L")
            _close(bel["z_lin"][i], b.z_lin, 1e-6, 1e-9, f"{tag} z_lin")
            S_ref = _cov(b.L)
            _close(Sig[i][0:6, 0:6], S_ref[0:6, 0:6], 0.0, 1e-6, f"{tag} pose covariance")  # north-star bar
            _close(Sig[i], S_ref, 1e-8, 0.0, f"{tag} covariance")
            # per-hypothesis ConditioningCert of the predict and fusion PSD projections: eigenvalue
            # extremes at the absolute accuracy of eigh (~1e-12 of the largest), near-null count exact
            for m, (name, ref) in enumerate((("predict", r["pred_cond"]), ("fusion", r["fusion_cond"]))):
                _close(hcond[i, m, 1], ref[1], 1e-10, 0.0, f"{tag} {name} eig_max")
                _close(hcond[i, m, 0], ref[0], 0.0, 1e-12 * ref[1], f"{tag} {name} eig_min")
                _close(hcond[i, m, 2], hcond[i, m, 1] / hcond[i, m, 0], 1e-15, 0.0, f"{tag} {name} cond")
                _close(hcond[i, m, 3], ref[3], 0.0, 0.0, f"{tag} {name} near-null count")
            # the full cert_vec of the bin, MF and planar projections (primitives.py:80-123)
            for b in range(stats.shape[1]):
                _cert6(pcert["bins"][i, b], r["moments"]["psd_certs"][b], f"{tag} bin {b} Sigma_p cert")
            _cert6(pcert["mf"][i], r["mf"]["psd_cert"], f"{tag} MF L_rot cert")
            _cert6(pcert["planar"][i], r["planar"]["psd_cert"], f"{tag} planar L_trans cert")
            _close(dPp[i], r["dPsi_proc"], 1e-8, 1e-18, f"{tag} dPsi_proc")
            _close(dPm[i], r["dPsi_meas"], 1e-8, 1e-18, f"{tag} dPsi_meas")
        # every hypothesis: the device covariance is the inverse of the device information matrix
        for i in range(H):
            _close(Sig[i], _cov(bel["L"][i]), 1e-8, 0.0, f"scan{k} hyp{i} Σ vs L")
        # barycenter combine over ALL hypotheses, from the GPU's per-hypothesis beliefs
        comb = O.hypothesis_barycenter(bel["L"], bel["h"], bel["z_lin"], weights, floor)
        c = pipe.combined()
        _close(c["L"], comb["L"], 1e-10, 0.0, f"scan{k} combined L")
        _close(c["h"], comb["h"], 1e-10, 1e-12, f"scan{k} combined h")
        _close(c["z_lin"], comb["z_lin"], 1e-10, 1e-12, f"scan{k} combined z_lin")
        _close(c["X_anchor"], bel["X_anchor"][0], 0.0, 0.0, f"scan{k} combined anchor = hypothesis 0")
        # the combined belief's ConditioningCert (hypothesis.py:186-202): eigenvalue extremes of the
        # projected barycenter (absolute accuracy ~1e-12 of the largest), near-null count exact
        pc = comb["psd_cert"]
        _close(c["eig_max"], pc[3], 1e-10, 0.0, f"scan{k} combined eig_max")
        _close(c["eig_min"], pc[2], 0.0, 1e-12 * pc[3], f"scan{k} combined eig_min")
        _close(c["near_null"], pc[5], 0.0, 0.0, f"scan{k} combined near-null count")
        Sc = _cov(comb["L"])
        _close(_cov(c["L"])[0:6, 0:6], Sc[0:6, 0:6], 0.0, 1e-6, f"scan{k} combined pose covariance")
        _cert6(pcert["barycenter"], pc, f"scan{k} barycenter projection cert")
        # IW apply from the GPU's per-hypothesis statistics of ALL hypotheses
        aP = np.einsum("k,kabc->abc", weights, dPp)
        aM = np.einsum("k,kabc->abc", weights, dPm)
        wp = float(min(1, k))
        nu_p, Psi_p, _ = O.iw_process_apply(iw0["nu_proc"], iw0["Psi_proc"], wp * aP, wp * np.full(7, weights.sum()))
        nu_m, Psi_m, _ = O.iw_meas_apply(iw0["nu_meas"], iw0["Psi_meas"], aM, weights.sum() * np.array([1.0, 1.0, 0.0]))
        iw = pipe.get_iw()
        _close(iw["nu_proc"], nu_p, 1e-12, 0, f"scan{k} nu_proc")
        _close(iw["Psi_proc"], Psi_p, 1e-9, 1e-20, f"scan{k} Psi_proc")
        _close(iw["nu_meas"], nu_m, 1e-12, 0, f"scan{k} nu_meas")
        _close(iw["Psi_meas"], Psi_m, 1e-9, 1e-20, f"scan{k} Psi_meas")
        _close(iw["Q"], O.iw_process_Q(nu_p, Psi_p), 1e-9, 1e-20, f"scan{k} Q")
        cp = O.iw_process_block_certs(iw0["Psi_proc"], wp * aP)
        cm = O.iw_meas_block_certs(iw0["Psi_meas"], aM)
        for b in range(7):
            _cert6(pcert["iw_proc"][b], cp[b], f"scan{k} process-IW block {b} cert")
        for b in range(3):
            _cert6(pcert["iw_meas"][b], cm[b], f"scan{k} measurement-IW block {b} cert")
        _cert6(pcert["Q"], O.iw_process_Q_cert(nu_p, Psi_p), f"scan{k} Q projection cert")
        # map: hypothesis 0's pushforward increment on the forgotten map (backend_node.py:2081-2083)
        if res0 is not None:
            mp = pipe.get_map()
            _close(mp["map"], cases.map_to_record(O.map_forget_and_add(mapst, res0["map_inc"])), 1e-8, 1e-12,
                   f"scan{k} map")
        # full-size properties of every hypothesis: Σ_b N_b = Σ w_deskew (bin cert [6]), finite
        np.testing.assert_allclose(stats[:, :, 0].sum(1), bcert[:, 6], rtol=1e-12)
        assert np.all(np.isfinite(bel["L"])) and np.all(np.isfinite(diag))
    return pipe


def test_c2_full_scan_64k_single_hypothesis(ctx):
    """C2: 65,536 points, H = 1, three scans with map and IW feedback (the fused kernel at its
    automatic geometry: one 256-point iteration per workgroup at H = 1)."""
    case = cases.build(H=1, n_az=4096, n_scans=3, io="computed")
    _run_and_compare(ctx, case, 1, case["n"], [0], 3, True)


def test_c3_bench_workload_matches_oracle(ctx):
    """C3 = the bench.py step: 65,536 points x 256 hypotheses, IMU/odom branch computed, 16
    iterations per fused workgroup, H = 256 combine, two scans (the second with the process-IW
    update and the cached posterior factorisation)."""
    case = cases.build(H=256, n_az=4096, n_scans=2, io="computed")
    _run_and_compare(ctx, case, 256, case["n"], [0, 1, 127, 255], 2, True)


TURNED_YAWS = [np.pi - 0.02, -np.pi + 0.02, 2.5, np.pi - 0.02]


def test_c3_turned_around_matches_oracle(ctx):
    """C3 (65,536 points x 256 hypotheses, IMU/odom branch computed, two scans) for a robot that
    has turned around: the world frame (warm-up map, odometry) is turned by π - 0.02, and the
    anchors' yaws cycle over π - 0.02, -π + 0.02, 2.5 rad with N(0, 0.1²) roll/pitch. Every
    world pose, recompose, anchor drift, ξ_body, MF δ and odom residual then goes through the Lie
    maps at large angles, and hypotheses cross the ±π cut of the rotation vector
    (se3_jax.py:304-366). Same bars as C3; sampled hypotheses cover every yaw."""
    case = cases.build(H=256, n_az=4096, n_scans=2, io="computed", yaw0=np.pi - 0.02, hyp_yaws=TURNED_YAWS,
                       tilt=0.1)
    assert np.any(np.abs(np.linalg.norm(case["hyp"]["X_anchor"][:, 3:6], axis=1)) > 3.1)
    _run_and_compare(ctx, case, 256, case["n"], [0, 1, 2, 3, 254], 2, True)


def test_c5_shape_matches_oracle(ctx):
    """C5 shape on one GPU: 131,072 points budgeted to 65,536 (stride 2) x 1024 hypotheses."""
    case = cases.build(H=1024, n_az=8192, n_scans=1, io="computed", cap=65536)
    _run_and_compare(ctx, case, 1024, 65536, [0, 511, 1023], 1, True)


def test_c3_inscan_certs_match_oracle(ctx):
    """C3 with the in-scan ConditioningCerts on (gc_certs.hip, computed inside the scan right after the
    evidence kernel): every bar of the C3 test, the per-hypothesis predict / fusion certificates among
    them, now read from the scan itself."""
    case = cases.build(H=256, n_az=4096, n_scans=1, io="computed")
    pipe = _pipeline(case, ctx, 256, case["n"], True)
    pipe.set_inscan_certs(True)
    _run_and_compare(ctx, case, 256, case["n"], [0, 1, 255], 1, True, pipe=pipe)


def _c5_with_map(ctx, cap):
    """C5 at its full size on one GPU: 131,072-point scans, H = 1024, the IMU/odom branch computed
    and the 1,048,576-slot PrimitiveMap attached (the in-scan update inside every scan). Sampled
    hypotheses against the oracle at the C3 bars, and the whole map against the oracle's
    scan_map_update after the scan (test_gpu_scanmap.py's bars)."""
    from test_gpu_scanmap import _check_scan, _map
    case = cases.build(H=1024, n_az=8192, n_scans=1, io="computed", cap=cap)
    pipe = _pipeline(case, ctx, 1024, cap, True)
    M, voxel = 1 << 20, 0.1
    dm = _map(ctx, M, 5)
    pipe.attach_primitive_map(dm, voxel)
    touched = []

    def before(k):
        return dm.download(), pipe.get_iw()

    def after(k, x):
        touched.append(_check_scan(pipe, dm, x[0], case["scans"][k], k, cap, M, voxel, x[1]))

    _run_and_compare(ctx, case, 1024, cap, [0, 511, 1023], 1, True, pipe=pipe, hooks=(before, after))
    assert touched and touched[0] > 1000, touched
    pipe.close()


def test_c5_with_map_matches_oracle(ctx):
    """C5 budgeted (stride 2: 131,072 -> 65,536 points) with the 1M-slot map attached."""
    _c5_with_map(ctx, 65536)


def test_c5_dense_with_map_matches_oracle(ctx):
    """C5 dense: every one of the 131,072 points kept (cap = 131,072, no stride) with the 1M-slot map."""
    _c5_with_map(ctx, 131072)


def test_c3_is_bit_reproducible(ctx):
    """Two pipelines fed the same C3 inputs agree bit for bit (no float atomics; fixed-order
    cross-workgroup reductions)."""
    case = cases.build(H=256, n_az=4096, n_scans=1, io="computed")
    outs = []
    for _ in range(2):
        pipe = _pipeline(case, ctx, 256, case["n"], True)
        s = case["scans"][0]
        pipe.stage_scan(0, s)
        pipe.run_scan(0, s, 0)
        ctx.sync()
        b = pipe.get_beliefs()
        outs.append((b["L"], b["h"], b["X_anchor"], pipe.combined()["L"], pipe.get_iw()["Psi_meas"],
                     pipe.get_map()["map"], pipe.bin_stats()[0]))
        pipe.close()
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


def _every_hypothesis(ctx, name, H, n_az, cap):
    """The first scan of a config for ALL its hypotheses against tests/golden/<name>_all.npz, the oracle's
    result for every hypothesis from the case's initial state (tests/golden/make_c3_all.py;
    tests/test_c3_fixture.py pins the fixtures to the inputs and the current oracle). The C3 test's bars:
    world pose, anchor and the pose block of Σ within 1e-6 abs (north star), z_lin 1e-6 rel, ξ_body
    1e-9 rel, α and the excitation-free β to 1e-12 / 1e-10 abs, T 1e-7 rel, cond_pose6 1e-6 rel."""
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"{name}_all.npz"))
    case = cases.build(H=H, n_az=n_az, n_scans=1, io="computed", cap=cap)
    n_cap = case["n"]
    pipe = _pipeline(case, ctx, H, n_cap, True)
    s = case["scans"][0]
    pipe.stage_scan(0, s)
    pipe.run_scan(0, s, 0)
    ctx.sync()
    diag, bel = pipe.hyp_diag(), pipe.get_beliefs()
    _, _, Sig = pipe.hyp_stats()
    _, _, xi = pipe.bin_stats()
    _close(diag[:, 0:6], g["pose"], 0.0, 1e-6, f"{name} every hypothesis: world pose")
    _close(bel["X_anchor"], g["X_anchor"], 0.0, 1e-6, f"{name} every hypothesis: X_anchor")
    _close(Sig[:, 0:6, 0:6], g["Sigma_pose"], 0.0, 1e-6, f"{name} every hypothesis: pose covariance")
    sc = g["scalars"]  # [alpha, beta, T, cond6]
    _close(diag[:, 8], sc[:, 0], 0.0, 1e-12, f"{name} every hypothesis: alpha")
    _close(diag[:, 7], sc[:, 1], 0.0, 1e-10, f"{name} every hypothesis: beta")
    for i in range(H):
        _close(bel["z_lin"][i], g["z_lin"][i], 1e-6, 1e-9, f"{name} hyp{i} z_lin")
        _close(xi[i], g["xi_body"][i], 1e-9, 1e-12, f"{name} hyp{i} xi_body")
        _close(diag[i, 6], sc[i, 2], 1e-7, 1e-10, f"{name} hyp{i} T")
        _close(diag[i, 13], sc[i, 3], 1e-6, 0.0, f"{name} hyp{i} cond_pose6")
    pipe.close()


def test_c3_every_hypothesis_matches_fixture(ctx):
    """C3 (the bench workload): all 256 hypotheses of the first scan (the other C3 tests run the oracle
    on 4-5 samples per scan)."""
    _every_hypothesis(ctx, "c3", 256, 4096, None)


def test_c5_every_hypothesis_matches_fixture(ctx):
    """C5 shape (131,072 points budgeted to 65,536, stride 2): all 1024 hypotheses of the first scan."""
    _every_hypothesis(ctx, "c5", 1024, 8192, 65536)
