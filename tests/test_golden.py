"""Committed golden vectors (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces its frozen outputs (guards the restatement against drift).
GPU: the HIP path reproduces the frozen outputs directly, oracle out of the loop. Tolerances
are the parity bars of tests/test_gpu_points.py / test_gpu_pipeline.py: integer contracts
bit-exact; pose within 1e-6 abs (north star); the rest relative, per assertion.
"""

import os

import numpy as np
import pytest

from oracle import cases
from oracle import gc_oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PIPE = dict(H=3, n_az=128, n_scans=2)


def _load(name):
    with np.load(os.path.join(GOLD, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


# ------------------------------------------------------------------------------- CPU (oracle)
def test_oracle_reproduces_ops_golden():
    g = _load("ops.npz")
    bud = O.point_budget_resample(g["in_pts"], g["in_t"], g["in_w"], None, None, int(g["in_cap"]))
    np.testing.assert_array_equal(bud["indices"], g["budget_indices"])
    np.testing.assert_array_equal(bud["points"], g["budget_points"])
    assert _rel(bud["weights"], g["budget_weights"]) < 1e-14
    p, w, _ = O.deskew_constant_twist(bud["points"], bud["timestamps"], bud["weights"], float(g["in_t0"]),
                                      float(g["in_t1"]), g["in_xi"])
    assert _rel(p, g["deskew_points"]) < 1e-13 and _rel(w, g["deskew_weights"]) < 1e-13
    sa = O.bin_soft_assign(g["dirs"], g["bins"])
    np.testing.assert_array_equal(sa["bin_index"], g["bin_index"])
    assert np.max(np.abs(sa["resp"] - g["resp"])) < 1e-15
    mm = O.scan_bin_moment_match(g["deskew_points"], g["in_covs"], g["deskew_weights"], g["resp"], g["in_lam"],
                                 g["origin"])
    for k in ("N", "s_dir", "S_dir_scatter", "p_bar", "Sigma_p", "kappa"):
        assert _rel(mm[k], g["mm_" + k]) < 1e-12, k
    assert _rel(O.kappa_batch(g["in_R_bar"]), g["kappa"]) < 1e-14
    for i, M in enumerate(g["in_psd_in"]):
        Mp, c = O.psd_project(M)
        assert _rel(Mp, g["psd_out"][i]) < 1e-13


def test_oracle_reproduces_pipeline_golden():
    g = _load("pipeline.npz")
    case = cases.build(**PIPE)
    from tests.golden.make_golden import digest
    keys = ("points", "timestamps", "weights", "imu_gyro", "imu_accel")
    dg = digest(*[case["scans"][k][key] for k in range(PIPE["n_scans"]) for key in keys])
    assert bytes(g["input_digest"]).hex() == dg, "synthetic scan generator changed: regenerate goldens"
    st = case["state"]
    for k, s in enumerate(case["scans"]):
        st, comb, res = O.process_scan(st, cases.scan_input(s), case["ios"], case["bins"], case["cfg"])
        assert np.max(np.abs(np.stack([r["pose"] for r in res]) - g[f"s{k}_pose"])) < 1e-12
        assert _rel(comb["L"], g[f"s{k}_comb_L"]) < 1e-11
        assert _rel(st.Psi_proc, g[f"s{k}_Psi_proc"]) < 1e-11
        assert _rel(cases.map_to_record(st.map), g[f"s{k}_map"]) < 1e-11


# --------------------------------------------------------------------------------- GPU (HIP)
@pytest.mark.gpu
def test_gpu_reproduces_ops_golden(ctx):
    from gcslam.ops import point_budget_resample
    from gcslam.ops.binning import bin_soft_assign_batch, scan_bin_moment_match_batch, unpack_bin_stats
    from gcslam.ops.deskew_constant_twist import deskew_batch
    from gcslam.ops.kappa import kappa_from_resultant_batch
    from gcslam.ops.primitives import domain_projection_psd_batch
    g = _load("ops.npz")
    res, _, _ = point_budget_resample(g["in_pts"], g["in_t"], g["in_w"], n_points_cap=int(g["in_cap"]), ctx=ctx)
    ns = g["budget_indices"].shape[0]
    np.testing.assert_array_equal(res.indices[:ns], g["budget_indices"])     # bit-exact selection
    np.testing.assert_array_equal(res.points, g["budget_points"])
    assert _rel(res.weights, g["budget_weights"]) < 1e-13
    pts, w, _ = deskew_batch(res.points, res.timestamps, res.weights, float(g["in_t0"]), float(g["in_t1"]),
                             g["in_xi"][None], ctx=ctx)
    assert np.max(np.abs(pts[0] - g["deskew_points"])) < 1e-12
    assert _rel(w[0], g["deskew_weights"]) < 1e-13
    resp, idx, cert = bin_soft_assign_batch(g["dirs"][None], g["bins"], 0.1, ctx=ctx)
    np.testing.assert_array_equal(idx[0], g["bin_index"])                    # bit-exact bin index
    assert np.max(np.abs(resp[0] - g["resp"])) < 1e-14
    assert abs(cert[0, 0] - g["avg_entropy"]) < 1e-9 and abs(cert[0, 1] - g["max_resp"]) < 1e-14
    stats, _ = scan_bin_moment_match_batch(g["deskew_points"][None], g["in_covs"][None], g["deskew_weights"][None],
                                           g["resp"][None], g["in_lam"][None], g["origin"], ctx=ctx)
    u = unpack_bin_stats(stats[0])
    for k, tol in (("N", 1e-10), ("s_dir", 1e-10), ("S_dir_scatter", 1e-10), ("p_bar", 1e-9),
                   ("Sigma_p", 1e-8), ("kappa", 1e-8)):
        assert _rel(u[k], g["mm_" + k]) < tol, k
    assert _rel(kappa_from_resultant_batch(g["in_R_bar"], ctx=ctx), g["kappa"]) < 1e-10
    Mp, _ = domain_projection_psd_batch(g["in_psd_in"], ctx=ctx)
    assert np.max(np.abs(Mp - g["psd_out"])) < 1e-9


@pytest.mark.gpu
def test_gpu_reproduces_pipeline_golden(ctx):
    from gcslam.pipeline import BatchedScanPipeline, PipelineConfig
    g = _load("pipeline.npz")
    case = cases.build(**PIPE)
    H = PIPE["H"]
    pipe = BatchedScanPipeline(H, case["n"], PipelineConfig(n_points_cap=case["n"]), ctx=ctx)
    hy = case["hyp"]
    pipe.set_beliefs(hy["X_anchor"], hy["z_lin"], hy["L"], hy["h"], hy["stamp"])
    pipe.set_weights(hy["weights"])
    pipe.set_io_evidence(*case["io"])
    pipe.set_iw(*case["iw"])
    pipe.set_map(case["map_record"])
    for k, s in enumerate(case["scans"]):
        pipe.stage_scan(0, s)
        pipe.run_scan(0, s, k)
        ctx.sync()
        diag = pipe.hyp_diag()
        assert np.max(np.abs(diag[:, 0:6] - g[f"s{k}_pose"])) < 1e-6            # north-star bar
        bel = pipe.get_beliefs()
        assert np.max(np.abs(bel["X_anchor"] - g[f"s{k}_X_anchor"])) < 1e-6
        assert _rel(bel["L"], g[f"s{k}_L"]) < 1e-8
        c = pipe.combined()
        assert _rel(c["L"], g[f"s{k}_comb_L"]) < 1e-8
        iw = pipe.get_iw()
        assert _rel(iw["Psi_proc"], g[f"s{k}_Psi_proc"]) < 1e-7
        assert _rel(iw["Psi_meas"], g[f"s{k}_Psi_meas"]) < 1e-7
        assert _rel(pipe.get_map()["map"], g[f"s{k}_map"]) < 1e-8
