"""The split a2 predict (csrc/gc_belief.hip) restated on the oracle (CPU): the predicted moments the
bins need, μ_inc = (L_pred + ε_l I)⁻¹ h_pred and σ_warp² = (L_pred + ε_l I)⁻¹[15, 15] with L_pred =
(Σ' + ε_l I)⁻¹ (predict.py:43-98; pipeline.py:436-453), equal K⁻¹ μ and (K⁻¹ (Σ' + ε_l I))[15, 15] with
K = I + ε_l (Σ' + ε_l I), a matrix within ε_l ‖Σ'‖ of the identity. The device takes the second form
(a Richardson iteration on one wave) and forms L_pred beside the bins; this pins the identity on the
oracle's own posteriors (cond(Σ') ~ 1e13 at the second scan) to the rounding of the reference route."""

import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import cases  # noqa: E402
from oracle import gc_oracle as O  # noqa: E402


def _richardson(S, b, eps):
    """wave_lift_iterate's iteration: x <- b - B x from x = b, B = eps (S_sym + eps I), ceil(56 ln2 / -ln r) steps."""
    B = eps * (0.5 * (S + S.T) + eps * np.eye(S.shape[0]))
    r = np.abs(B).sum(1).max()
    assert r <= 0.25
    x = b.copy()
    for _ in range(int(math.ceil(38.816242111356935 / -math.log(r)))):
        x = b - B @ x
    return x


def test_predicted_moments_from_sigma_match_the_factorised_route():
    case = cases.build(H=3, n_az=256, n_scans=2, io="computed")
    st = case["state"]
    Q = O.iw_process_Q(st.nu_proc, st.Psi_proc)
    Sga = (O.iw_meas_mode(st.nu_meas, st.Psi_meas, 0), O.iw_meas_mode(st.nu_meas, st.Psi_meas, 1))
    md = O.map_derived(st.map)
    e = O.EPS_LIFT
    conds = []
    for k in range(3):
        b = st.beliefs[k]
        for scan in case["scans"]:
            sc = cases.scan_input(scan)
            bpred, _ = O.predict_diffusion(b, Q, sc.dt_sec)           # the reference route
            mu_ref = O.chol_solve_lifted(bpred.L, bpred.h)[0]
            s_ref = O.chol_inverse_lifted(bpred.L)[0][15, 15]
            mu = O.chol_solve_lifted(b.L, b.h)[0]                      # the split route
            cov = O.chol_inverse_lifted(b.L)[0]
            ef = math.exp(-2.0 * O.OU_LAMBDA * sc.dt_sec)
            dc = (1.0 - ef) / (2.0 * O.OU_LAMBDA + O.F64_EPS)
            S = ef * cov + dc * Q
            mu_new = _richardson(S, mu, e)
            col = 0.5 * (S[:, 15] + S[15, :]) + e * np.eye(22)[:, 15]
            s_new = _richardson(S, col, e)[15]
            conds.append(np.linalg.cond(S))
            assert np.max(np.abs(mu_new - mu_ref)) <= 1e-14 * max(np.max(np.abs(mu_ref)), 1e-300) + 1e-17
            assert abs(s_new - s_ref) <= 1e-13 * s_ref
            b = O.scan_hypothesis(b, sc, Q, None, st.map, md, case["bins"], case["cfg"], Sga)["belief"]
    assert max(conds) > 1e10  # the second scan's Σ' is ill-conditioned: the identity holds there too
