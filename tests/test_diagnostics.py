"""Diagnostics tape / manifest / TUM export: MinimalScanTape and DiagnosticsLog
(backend/diagnostics.py:18-329) round trips in both of the reference's file formats, the TUM line
format (backend_node.py:1257-1260, 2287-2293), and a tape filled from the device pipeline against
the oracle's values for the same scan (GPU)."""

import numpy as np
import pytest

from oracle import gc_oracle as O


def _tape(i):
    from gcslam.diagnostics import MinimalScanTape
    rng = np.random.default_rng(i)
    kw = dict(scan_number=i, timestamp=10.0 + i, dt_sec=0.1, n_points_raw=65536, n_points_budget=8192,
              fusion_alpha=1.0, cond_pose6=rng.uniform(1, 100), conditioning_number=3.0, eigmin_pose6=0.5,
              L_pose6=rng.normal(size=(6, 6)), total_trigger_magnitude=rng.uniform(), cert_exact=False,
              cert_frobenius_applied=True, cert_n_triggers=3, support_ess_total=100.0, support_frac=0.9,
              mismatch_nll_per_ess=0.1, mismatch_directional_score=1.0, excitation_dt_effect=0.2,
              excitation_extrinsic_effect=0.3, influence_psd_projection_delta=0.0, influence_mass_epsilon_ratio=1e-12,
              influence_anchor_drift_rho=0.1, influence_dt_scale=0.8, influence_extrinsic_scale=0.7,
              influence_trust_alpha=1.0, influence_power_beta=0.5, overconfidence_excitation_total=1.0,
              overconfidence_ess_to_excitation=0.0, overconfidence_cond_to_support=0.0,
              overconfidence_dt_asymmetry=0.1, overconfidence_z_to_xy_ratio=0.2, t_total_ms=1.6)
    return MinimalScanTape(**kw)


def _same(a, b):
    import dataclasses
    for f in dataclasses.fields(a):
        va, vb = getattr(a, f.name), getattr(b, f.name)
        if f.name == "L_pose6":
            assert np.array_equal(va, vb)
        else:
            assert va == vb and type(va) is type(vb), (f.name, va, vb)


def test_tape_jsonl_and_npz_round_trip(tmp_path):
    from gcslam.diagnostics import DiagnosticsLog
    log = DiagnosticsLog(run_id="r1", start_time=5.0)
    for i in range(4):
        log.append_tape(_tape(i))
    log.save_jsonl(str(tmp_path / "d.jsonl"))
    log.save_npz(str(tmp_path / "d.npz"))
    for back in (DiagnosticsLog.load_jsonl(str(tmp_path / "d.jsonl")), DiagnosticsLog.load_npz(str(tmp_path / "d.npz"))):
        assert back.run_id == "r1" and back.total_scans == 4
        for a, b in zip(log.tape, back.tape):
            _same(a, b)
    # reference key names in the npz (diagnostics.py:216-222) and the loader defaults for absent keys
    z = np.load(str(tmp_path / "d.npz"))
    assert {"scan_numbers", "timestamps", "dt_secs", "L_pose6"} <= set(z.files) and str(z["format"]) == "minimal_tape"
    d = log.tape[0].to_dict()
    for k in ("cert_exact", "influence_dt_scale", "t_map_update_ms"):
        d.pop(k)
    from gcslam.diagnostics import MinimalScanTape
    e = MinimalScanTape.from_dict(d)
    assert e.cert_exact is True and e.influence_dt_scale == 1.0 and e.t_map_update_ms == 0.0
    DiagnosticsLog().save_npz(str(tmp_path / "e.npz"))
    assert DiagnosticsLog.load_npz(str(tmp_path / "e.npz")).total_scans == 0


def test_tum_writer_format(tmp_path):
    from gcslam.diagnostics import TumTrajectoryWriter, runtime_manifest
    w = TumTrajectoryWriter(str(tmp_path / "traj.tum"))
    w.write(12.5, [1.0, 2.0, 0.5, 0.0, 0.0, np.pi / 2])
    w.write(12.6, [0.0, 0.0, 0.0, 0.0, 0.0, 0.0])
    w.close()
    lines = open(tmp_path / "traj.tum").read().splitlines()
    assert lines[0] == "# timestamp x y z qx qy qz qw"
    f = [float(x) for x in lines[1].split()]
    assert lines[1].split()[0] == "12.500000000" and np.allclose(f[1:4], [1, 2, 0.5])
    assert np.allclose(f[4:], [0, 0, np.sin(np.pi / 4), np.cos(np.pi / 4)], atol=1e-6)
    assert lines[2].endswith("0.000000 0.000000 0.000000 1.000000")
    m = runtime_manifest()
    assert m["D_Z"] == 22 and m["backends"]["sinkhorn_backend"] == "unbalanced_fixed_k"


@pytest.mark.gpu
def test_gpu_tape_from_pipeline_matches_oracle(ctx, tmp_path):
    from gcslam.diagnostics import DiagnosticsLog, tape_from_pipeline
    from gcslam.pipeline import BatchedScanPipeline, PipelineConfig
    from oracle import cases
    case = cases.build(H=3, n_az=256, n_scans=1)
    s = case["scans"][0]
    pipe = BatchedScanPipeline(3, case["n"], PipelineConfig(n_points_cap=case["n"]), ctx=ctx)
    hy = case["hyp"]
    pipe.set_beliefs(hy["X_anchor"], hy["z_lin"], hy["L"], hy["h"], hy["stamp"])
    pipe.set_weights(hy["weights"])
    pipe.set_io_evidence(*case["io"])
    pipe.set_iw(*case["iw"])
    pipe.set_map(case["map_record"])
    pipe.stage_scan(0, s)
    pipe.run_scan(0, s, case["state"].scan_count)
    ctx.sync()
    n = case["n"]
    st, comb, res = O.process_scan(case["state"], cases.scan_input(s), case["ios"], case["bins"], case["cfg"])
    log = DiagnosticsLog(run_id="gpu")
    for h in range(3):
        t = tape_from_pipeline(pipe, 0, s["scan_end"], 0.1, n, n, hyp=h)
        r = res[h]
        assert abs(t.fusion_alpha - r["alpha"]) < 1e-12 and abs(t.influence_power_beta - r["beta"]) < 1e-10
        assert abs(t.cond_pose6 - r["cond6"]) <= 1e-6 * r["cond6"]
        assert abs(t.eigmin_pose6 - r["eigmin6"]) <= 1e-7 * r["eigmin6"] + 1e-12
        assert np.allclose(t.L_pose6, r["L_ev"][0:6, 0:6], rtol=1e-8, atol=1e-10)
        assert abs(t.total_trigger_magnitude - r["T"]) <= 1e-8 * abs(r["T"]) + 1e-10
        log.append_tape(t)
    log.save_jsonl(str(tmp_path / "g.jsonl"))
    assert DiagnosticsLog.load_jsonl(str(tmp_path / "g.jsonl")).total_scans == 3


def test_cert_summary_of_the_bin_path_wiring():
    """cert_n_triggers / mismatch_directional_score of aggregate_certificates over the wiring's cert
    list: 23 trigger names over 25 certs; only the vMF cert's R̄ varies (odom, gyro and preint
    factor certs score 0, the rest keep the default 1)."""
    from gcslam.diagnostics import BIN_PATH_CERTS, TAPE_NOT_COMPUTED, cert_summary
    assert TAPE_NOT_COMPUTED == () and len(BIN_PATH_CERTS) == 25
    n, d = cert_summary(0.4)
    assert n == 23 and abs(d - (21.0 + 0.4) / 25.0) < 1e-15


@pytest.mark.gpu
def test_gpu_tape_certificate_summary_fields(ctx):
    """The four certificate-summary fields on a device scan with the IMU/odom branch computed:
    directional score from the branch's vMF R̄ (checked against the oracle), the FusionScale
    sentinels ESS/(excitation + ε) and cond/(support + ε) (fusion.py:121-130)."""
    from gcslam.diagnostics import tape_from_pipeline
    from gcslam.pipeline import BatchedScanPipeline, PipelineConfig
    from oracle import cases
    case = cases.build(H=2, n_az=256, n_scans=1, io="computed")
    s = case["scans"][0]
    pipe = BatchedScanPipeline(2, case["n"], PipelineConfig(n_points_cap=case["n"]), ctx=ctx)
    hy = case["hyp"]
    pipe.set_beliefs(hy["X_anchor"], hy["z_lin"], hy["L"], hy["h"], hy["stamp"])
    pipe.set_weights(hy["weights"])
    pipe.set_io_mode(True)
    pipe.set_iw(*case["iw"])
    pipe.set_map(case["map_record"])
    pipe.stage_scan(0, s)
    pipe.run_scan(0, s, 0)
    ctx.sync()
    st, comb, res = O.process_scan(case["state"], cases.scan_input(s), None, case["bins"], case["cfg"])
    d = pipe.hyp_diag()
    for h in range(2):
        t = tape_from_pipeline(pipe, 0, s["scan_end"], 0.1, case["n"], case["n"], hyp=h)
        rbar = res[h]["io_parts"]["imu"]["Rbar"]
        assert t.cert_n_triggers == 23
        assert abs(t.mismatch_directional_score - (21.0 + rbar) / 25.0) < 1e-12
        assert t.overconfidence_ess_to_excitation == d[h, 14] / (d[h, 37] + 1e-12)
        assert abs(t.overconfidence_cond_to_support - res[h]["cond6"] / (d[h, 36] + 1e-12)) <= 1e-6 * abs(
            t.overconfidence_cond_to_support)
