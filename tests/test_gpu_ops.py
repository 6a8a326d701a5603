"""GPU parity of the per-operator entries (a2, a3, a7-a12, a14-a16, world pose) against the CPU
oracle on seeded inputs, called through the reference-signature mirror (gcslam.ops) and the
batched C entries. Tolerances per assertion: f64 ulps from ocml vs libm, Jacobi vs LAPACK eigh,
parallel vs sequential sums; poses within the north-star 1e-6 abs (here far tighter)."""

import numpy as np
import pytest

from oracle import gc_oracle as O

pytestmark = pytest.mark.gpu

D = 22


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def _spd(rng, scale=1.0):
    A = rng.normal(size=(D, D))
    return scale * (A @ A.T / D + 0.1 * np.eye(D))


def _belief(rng, k=0):
    from gcslam.belief import BeliefGaussianInfo
    L = _spd(rng, 10.0 ** (k % 3))
    return BeliefGaussianInfo("GC-RIGHT-01", f"a{k}", rng.normal(0, 0.3, 6), 100.0 + k, rng.normal(0, 0.05, D), L,
                              rng.normal(0, 1.0, D))


def _ob(b):
    return O.Belief(b.X_anchor.copy(), b.z_lin.copy(), b.L.copy(), b.h.copy(), b.stamp_sec)


def test_world_pose_and_mean(ctx):
    from gcslam.belief import world_pose_batch
    rng = np.random.default_rng(11)
    bs = [_belief(rng, k) for k in range(5)]
    pose, mean = world_pose_batch(bs, ctx=ctx)
    for k, b in enumerate(bs):
        ob = _ob(b)
        assert _rel(mean[k], O.mean_increment(ob)) < 1e-10
        assert np.max(np.abs(pose[k] - O.world_pose(ob))) < 1e-12


@pytest.mark.parametrize("dt", [0.1, 0.0, 3.7])
def test_predict_diffusion(ctx, dt):
    from gcslam.ops import predict_diffusion
    rng = np.random.default_rng(12)
    b = _belief(rng)
    Q = _spd(rng, 1e-3)
    out, cert, eff = predict_diffusion(b, Q, dt, ctx=ctx)
    ref, rc = O.predict_diffusion(_ob(b), Q, dt)
    assert _rel(out.L, ref.L) < 1e-9 and _rel(out.h, ref.h) < 1e-9
    assert out.stamp_sec == b.stamp_sec + dt
    assert abs(cert.influence.psd_projection_delta - rc["psd_delta"]) < 1e-9 * max(1.0, np.abs(ref.L).max())
    assert abs(cert.conditioning.eig_min - rc["cond"][0]) <= 1e-7 * rc["cond"][0]
    assert abs(cert.conditioning.eig_max - rc["cond"][1]) <= 1e-9 * rc["cond"][1]
    assert abs(eff.predicted - rc["trace_cov"]) <= 1e-10 * rc["trace_cov"]
    assert abs(cert.total_trigger_magnitude() - rc["trig"]) < 1e-9


def test_predict_projects_indefinite_q(ctx):
    """A non-PSD process noise exercises the clamp path of both projections."""
    from gcslam.ops.predict import predict_diffusion_batch
    rng = np.random.default_rng(13)
    b = _belief(rng)
    Q = -_spd(rng, 1.0)
    Lp, hp, c = predict_diffusion_batch(b.L[None], b.h[None], Q, 5.0, ctx=ctx)
    ref, rc = O.predict_diffusion(_ob(b), Q, 5.0)
    # the clamped covariance eigenvalues sit at eps_psd = 1e-12, so L' ~ 1e12 scale: condition-limited
    assert _rel(Lp[0], ref.L) < 1e-6 and c[0, 1] > 0 and abs(c[0, 1] - rc["psd_delta"]) <= 1e-5 * rc["psd_delta"]


def test_window_weights_and_preintegration(ctx):
    from gcslam import synth
    from gcslam.ops import preintegrate_imu_relative_pose_jax, smooth_window_weights
    from gcslam.ops.imu_preintegration import preintegrate_imu_batch
    s = synth.make_scan(3, n_az=64)
    t, g, a = s["imu_stamps"], s["imu_gyro"], s["imu_accel"]
    w = smooth_window_weights(t, s["scan_start"], s["scan_end"], 0.02, ctx=ctx)
    np.testing.assert_allclose(w, O.smooth_window_weights(t, s["scan_start"], s["scan_end"], 0.02), rtol=1e-14,
                               atol=1e-300)
    rng = np.random.default_rng(14)
    H = 3
    r0 = rng.normal(0, 0.2, (H, 3)); bg = rng.normal(0, 1e-3, (H, 3)); ba = rng.normal(0, 1e-2, (H, 3))
    out = preintegrate_imu_batch(t, g, a, w, r0, bg, ba, ctx=ctx)
    for k in range(H):
        ref = O.preintegrate(t, g, a, w, r0[k], bg[k], ba[k])
        assert np.max(np.abs(out[k, 0:6] - ref["delta_pose"])) < 1e-11
        assert np.max(np.abs(out[k, 6:15].reshape(3, 3) - ref["delta_R"])) < 1e-13
        assert _rel(out[k, 18:21], ref["delta_v"]) < 1e-11
        assert abs(out[k, 21] - ref["ess"]) < 1e-12 * ref["ess"]
        for j, key in ((22, "a_body_mean"), (25, "a_world_nog_mean"), (28, "a_world_mean")):
            assert _rel(out[k, j:j + 3], ref[key]) < 1e-11, key
        assert abs(out[k, 31] - ref["dt_eff_sum"]) < 1e-13
    dp, dR, p_b, v_b, ess, *_ = preintegrate_imu_relative_pose_jax(t, g, a, w, r0[0], bg[0], ba[0],
                                                                   (0.0, 0.0, -9.81), ctx=ctx)
    assert np.max(np.abs(dp - O.preintegrate(t, g, a, w, r0[0], bg[0], ba[0])["delta_pose"])) < 1e-11


def test_imu_meas_iw_suffstats(ctx):
    from gcslam import synth
    from gcslam.ops.imu_preintegration import imu_meas_iw_suffstats_batch
    s = synth.make_scan(4, n_az=64)
    g, a = s["imu_gyro"], s["imu_accel"]
    rng = np.random.default_rng(15)
    w = rng.uniform(0, 1, g.shape[0])
    H = 2
    bg, ba = rng.normal(0, 1e-3, (H, 3)), rng.normal(0, 1e-2, (H, 3))
    om, r0 = rng.normal(0, 0.1, (H, 3)), rng.normal(0, 0.2, (H, 3))
    out = imu_meas_iw_suffstats_batch(g, a, w, bg, ba, om, r0, 0.005, ctx=ctx)
    for k in range(H):
        assert _rel(out[k, 0], O.iw_meas_gyro_suffstats(g, w, bg[k], om[k], 0.005)) < 1e-10
        assert _rel(out[k, 1], O.iw_meas_accel_suffstats(r0[k], a, w, ba[k], 0.005)) < 1e-10


def _bins_case(rng, B=48):
    sN = rng.uniform(1, 50, B); mN = rng.uniform(1, 50, B)
    s_dir = rng.normal(size=(B, 3)) * sN[:, None] * 0.5
    m_dir = rng.normal(size=(B, 3)) * mN[:, None] * 0.5
    def scat(n):
        A = rng.normal(size=(B, 3, 3)) * 0.3
        return (A @ np.swapaxes(A, 1, 2)) * n[:, None, None]
    return sN, s_dir, scat(sN), mN, m_dir, scat(mN)


def test_matrix_fisher(ctx):
    from gcslam.belief import world_pose_batch
    from gcslam.ops import matrix_fisher_rotation_evidence
    rng = np.random.default_rng(16)
    b = _belief(rng)
    sN, s_dir, sS, mN, m_dir, mS = _bins_case(rng)
    res, cert, eff = matrix_fisher_rotation_evidence(b, s_dir, sS, sN, m_dir, mS, mN, ctx=ctx)
    pose = world_pose_batch([b], ctx=ctx)[0][0]
    ref = O.matrix_fisher(O.so3_exp(pose[3:6]), s_dir, sS, sN, m_dir, mS, mN)
    assert np.max(np.abs(res.R_mf - ref["R_mf"])) < 1e-12
    assert _rel(res.L_rot, ref["L_rot"]) < 1e-10 and _rel(res.h_rot, ref["h_rot"]) < 1e-9
    assert np.max(np.abs(res.delta_rot - ref["delta_rot"])) < 1e-12
    assert _rel(res.svd_singular_values, ref["svd"]) < 1e-12
    assert abs(cert.mismatch.nll_per_ess - ref["nll_per_ess"]) <= 1e-9 * ref["nll_per_ess"] + 1e-300
    for got, exp in ((res.map_scatter_metrics, ref["map_metrics"]), (res.scan_scatter_metrics, ref["scan_metrics"])):
        assert _rel(got.eigenvalues, exp["eigenvalues"]) < 1e-12
        # eigenvectors up to sign
        assert np.max(np.abs(np.abs(np.sum(got.eigenvectors * exp["eigenvectors"], axis=0)) - 1.0)) < 1e-10
        for k in ("linearity", "planarity", "sphericity", "anisotropy", "effective_rank"):
            assert abs(getattr(got, k) - exp[k]) < 1e-11, k


def test_planar_translation(ctx):
    from gcslam.belief import world_pose_batch
    from gcslam.ops import planar_translation_evidence
    rng = np.random.default_rng(17)
    b = _belief(rng)
    B = 48
    sN, _, _, mN, _, mS = _bins_case(rng, B)
    p_bar = rng.normal(0, 4, (B, 3)); c_map = p_bar + rng.normal(0, 0.1, (B, 3))
    A = rng.normal(size=(B, 3, 3)) * 0.1
    Sig_p = A @ np.swapaxes(A, 1, 2); Sig_c = Sig_p[::-1].copy()
    Npos = rng.uniform(1, 30, B)
    R_hat = O.so3_exp(rng.normal(0, 0.1, 3))
    res, cert, eff = planar_translation_evidence(b, p_bar, Sig_p, sN, c_map, Sig_c, Npos, mS, mN, R_hat, ctx=ctx)
    pose = world_pose_batch([b], ctx=ctx)[0][0]
    ref = O.planar_translation(pose[0:3], p_bar, Sig_p, sN, c_map, Sig_c, Npos, mS, mN, R_hat)
    assert _rel(res.t_wls, ref["t_wls"]) < 1e-10
    assert _rel(res.L_trans, ref["L_trans"]) < 1e-10 and _rel(res.h_trans, ref["h_trans"]) < 1e-9
    assert abs(res.xy_info_scale - ref["xy_info_scale"]) <= 1e-10 * ref["xy_info_scale"]
    assert abs(res.z_info_scale - ref["z_info_scale"]) <= 1e-9 * abs(ref["z_info_scale"]) + 1e-18


def test_excitation_and_fusion_scale(ctx):
    from gcslam.certificates import (CertBundle, ConditioningCert, ExcitationCert, InfluenceCert, MismatchCert,
                                     OverconfidenceCert, SupportCert)
    from gcslam.ops import apply_excitation_prior_scaling_jax, fusion_scale_from_certificates
    from gcslam.ops.excitation import excitation_scaling_batch
    rng = np.random.default_rng(18)
    Le, Lp, hp = _spd(rng), _spd(rng, 3.0), rng.normal(size=D)
    s, Lo, ho = excitation_scaling_batch(Le[None], Lp[None], hp[None], ctx=ctx)
    rL, rh, sdt, sex = O.excitation_scaling(Le, Lp, hp)
    assert abs(s[0, 0] - sdt) < 1e-15 and abs(s[0, 1] - sex) < 1e-15
    np.testing.assert_allclose(Lo[0], rL, rtol=1e-15, atol=0)
    np.testing.assert_allclose(ho[0], rh, rtol=1e-15, atol=0)
    L2, h2 = apply_excitation_prior_scaling_jax(Lp, hp, sdt, sex, ctx=ctx)
    np.testing.assert_allclose(L2, rL, rtol=1e-15, atol=0)
    ce = CertBundle.create_exact("GC-RIGHT-01", "a", conditioning=ConditioningCert(cond=123.0),
                                 support=SupportCert(ess_total=7.0, support_frac=0.9),
                                 excitation=ExcitationCert(dt_effect=0.3, extrinsic_effect=0.4),
                                 overconfidence=OverconfidenceCert(dt_asymmetry=0.6, z_to_xy_ratio=2.0),
                                 influence=InfluenceCert(power_beta=0.8), mismatch=MismatchCert(nll_per_ess=0.2))
    for amin, amax in ((1.0, 1.0), (0.1, 1.0)):
        r, c, _ = fusion_scale_from_certificates(ce, ce, alpha_min=amin, alpha_max=amax, ctx=ctx)
        assert abs(r.alpha - O.fusion_alpha(123.0, 7.0, 0.7, 0.6, 2.0, 0.8, 0.2, amin, amax)) < 1e-15


def test_info_fusion_additive(ctx):
    from gcslam.ops import info_fusion_additive
    rng = np.random.default_rng(19)
    b = _belief(rng)
    Le = _spd(rng) - 2.0 * np.eye(D)   # indefinite evidence: the projection clamps
    he = rng.normal(size=D)
    for alpha in (1.0, 0.4):
        post, cert, _ = info_fusion_additive(b, Le, he, alpha, ctx=ctx)
        rL, rh, rc = O.info_fusion_additive(b.L, b.h, Le, he, alpha)
        assert _rel(post.L, rL) < 1e-10 and _rel(post.h, rh) < 1e-14
        assert abs(cert.influence.psd_projection_delta - rc[0]) <= 1e-8 * max(rc[0], 1e-12)
        assert abs(cert.conditioning.eig_max - rc[3]) <= 1e-10 * rc[3]


def test_recompose_and_anchor_drift(ctx):
    from gcslam.ops import anchor_drift_update, pose_update_frobenius_recompose
    rng = np.random.default_rng(20)
    for k, T in enumerate((0.0, 0.37, 12.0)):
        b = _belief(rng, k)
        res, out, cert, _ = pose_update_frobenius_recompose(b, T, ctx=ctx)
        ref, rr = O.recompose(_ob(b), T)
        assert np.max(np.abs(out.X_anchor - ref.X_anchor)) < 1e-12
        assert _rel(out.z_lin, ref.z_lin) < 1e-10 and _rel(out.h, ref.h) < 1e-10
        assert abs(res.frobenius_strength - rr["frobenius_strength"]) < 1e-15
        assert cert.frobenius_applied == (T > 0)
        res2, out2, cert2, _ = anchor_drift_update(out, ctx=ctx)
        ref2, rd = O.anchor_drift(ref)
        assert abs(res2.rho - rd["rho"]) < 1e-10
        assert np.max(np.abs(out2.X_anchor - ref2.X_anchor)) < 1e-10
        assert _rel(out2.z_lin, ref2.z_lin) < 1e-9 and _rel(out2.h, ref2.h) < 1e-9


def test_inverse_wishart_ops(ctx):
    from gcslam.ops import (MeasurementNoiseIWState, ProcessNoiseIWState, measurement_noise_apply_suffstats_jax,
                            process_noise_iw_apply_suffstats_jax, process_noise_iw_suffstats_from_info_jax,
                            process_noise_state_to_Q_jax)
    rng = np.random.default_rng(21)
    Lq, Lp = _spd(rng), _spd(rng, 2.0)
    hq, hp = rng.normal(size=D), rng.normal(size=D)
    dP, dn = process_noise_iw_suffstats_from_info_jax(Lq, hq, Lp, hp, ctx=ctx)
    rP, rn = O.iw_process_suffstats(Lq, hq, Lp, hp)
    assert _rel(dP, rP) < 1e-9 and np.all(dn == rn)
    nu, Psi = O.iw_process_init()
    st, c = process_noise_iw_apply_suffstats_jax(ProcessNoiseIWState(nu, Psi), 0.3 * rP, 0.3 * rn, ctx=ctx)
    n2, P2, rc = O.iw_process_apply(nu, Psi, 0.3 * rP, 0.3 * rn)
    assert _rel(st.nu, n2) < 1e-14 and _rel(st.Psi, P2) < 1e-9
    # the projection delta here is ~1e-11 (eps-padded blocks): compare at 1e-13 absolute
    assert abs(c[1] - rc[1]) < 1e-12 and abs(c[0] - rc[0]) <= 1e-6 * rc[0] + 1e-13
    assert _rel(process_noise_state_to_Q_jax(st, ctx=ctx), O.iw_process_Q(n2, P2)) < 1e-9
    nuM, PsiM = O.iw_meas_init()
    A = rng.normal(size=(3, 3, 3)) * 1e-3
    dPM = A @ np.swapaxes(A, 1, 2)
    dnM = np.array([1.0, 1.0, 0.0])
    sm, cm = measurement_noise_apply_suffstats_jax(MeasurementNoiseIWState(nuM, PsiM), dPM, dnM, ctx=ctx)
    m2, Pm2, rcm = O.iw_meas_apply(nuM, PsiM, dPM, dnM)
    assert _rel(sm.nu, m2) < 1e-14 and _rel(sm.Psi, Pm2) < 1e-10


@pytest.mark.parametrize("K", [4, 7])
def test_hypothesis_barycenter(ctx, K):
    from gcslam.ops import hypothesis_barycenter_projection
    rng = np.random.default_rng(22 + K)
    bs = [_belief(rng, k) for k in range(K)]
    w = rng.uniform(0, 1, K); w[1] = 0.0
    floor = 0.01 / K
    res, cert, eff = hypothesis_barycenter_projection(bs, w, K_HYP=K, HYP_WEIGHT_FLOOR=floor, ctx=ctx)
    ref = O.hypothesis_barycenter(np.stack([b.L for b in bs]), np.stack([b.h for b in bs]),
                                  np.stack([b.z_lin for b in bs]), w, floor)
    out = res.belief_out
    assert _rel(out.L, ref["L"]) < 1e-10 and _rel(out.h, ref["h"]) < 1e-14 and _rel(out.z_lin, ref["z_lin"]) < 1e-14
    assert abs(res.floor_adjustment - ref["floor_adjustment"]) < 1e-15
    assert abs(eff.predicted - ref["spread"]) <= 1e-9 * ref["spread"]
    assert abs(cert.support.ess_total - ref["ess"]) <= 1e-13 * ref["ess"]
    assert abs(cert.support.support_frac - ref["support_frac"]) < 1e-15
    with pytest.raises(ValueError):
        hypothesis_barycenter_projection(bs, w, K_HYP=K + 1, ctx=ctx)


def _cond_fields(dev4, ref4, what):
    """ConditioningCert [eig_min, eig_max, cond, near_null_count] of a projection certified by the
    Cholesky shortcut + Sturm counts (gc_cond.h) against the oracle's eigh: eig_max 1e-10 relative,
    eig_min within 1e-12 of eig_max (the absolute accuracy of eigh), cond of the device's own extremes,
    the near-null count exact."""
    dev4, ref4 = np.asarray(dev4, np.float64), np.asarray(ref4, np.float64)
    assert abs(dev4[1] - ref4[1]) <= 1e-10 * ref4[1], (what, dev4, ref4)
    assert abs(dev4[0] - ref4[0]) <= 1e-12 * ref4[1], (what, dev4, ref4)
    assert abs(dev4[2] - dev4[1] / dev4[0]) <= 1e-15 * dev4[2], (what, dev4)
    if ref4[0] > 1e-5 * ref4[1]:
        assert abs(dev4[2] - ref4[2]) <= 1e-6 * ref4[2], (what, dev4, ref4)
    assert dev4[3] == ref4[3], (what, dev4, ref4)


def test_single_operator_certificates_on_the_shortcut(ctx):
    """predict_diffusion, info_fusion_additive and hypothesis_barycenter_projection with inactive clamps
    (SPD operands): the projections take the Cholesky-certified shortcut and the ConditioningCert comes
    from Sturm counts (no Jacobi sweep); every cert field against the oracle (projection delta 0 here vs
    the reference's rounding of V diag(λ) Vᵀ, ~1e-16 of the spectrum)."""
    from gcslam.ops import hypothesis_barycenter_projection, info_fusion_additive, predict_diffusion
    rng = np.random.default_rng(31)
    for k in range(3):
        b = _belief(rng, k)
        Q = _spd(rng, 1e-3)
        out, cert, _ = predict_diffusion(b, Q, 0.1, ctx=ctx)
        ref, rc = O.predict_diffusion(_ob(b), Q, 0.1)
        c = cert.conditioning
        _cond_fields([c.eig_min, c.eig_max, c.cond, c.near_null_count], rc["cond"], f"predict {k}")
        assert abs(cert.influence.psd_projection_delta - rc["psd_delta"]) <= 1e-12 * np.max(np.abs(ref.L))
        Le, he = _spd(rng, 3.0), rng.normal(size=D)
        post, cf, _ = info_fusion_additive(b, Le, he, 0.7, ctx=ctx)
        rL, rh, r6 = O.info_fusion_additive(b.L, b.h, Le, he, 0.7)
        c = cf.conditioning
        _cond_fields([c.eig_min, c.eig_max, c.cond, c.near_null_count], r6[2:6], f"fusion {k}")
        assert cf.influence.psd_projection_delta <= 1e-12 * r6[3] and abs(r6[0]) <= 1e-12 * r6[3]
        assert _rel(post.L, rL) < 1e-12
    K = 5
    bs = [_belief(rng, k) for k in range(K)]
    w = rng.uniform(0.1, 1, K)
    res, cb, _ = hypothesis_barycenter_projection(bs, w, K_HYP=K, HYP_WEIGHT_FLOOR=0.01 / K, ctx=ctx)
    ref = O.hypothesis_barycenter(np.stack([x.L for x in bs]), np.stack([x.h for x in bs]),
                                  np.stack([x.z_lin for x in bs]), w, 0.01 / K)
    c = cb.conditioning
    _cond_fields([c.eig_min, c.eig_max, c.cond, c.near_null_count], ref["psd_cert"][2:6], "barycenter")
    assert _rel(res.belief_out.L, ref["L"]) < 1e-12
