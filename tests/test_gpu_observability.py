"""Per-stage device timing, host accounting and the DeviceRuntimeCert of the batched pipeline.

Reference: MinimalScanTape.t_*_ms per stage (pipeline.py:383-394, :1560-1569), RuntimeCounters /
consume_runtime_counters (common/runtime_counters.py:19-108) surfaced as DeviceRuntimeCert
(backend_node.py:2182-2190). Timing must not change a single bit of the results.
"""

import numpy as np
import pytest

from oracle import cases
from test_gpu_configs import _pipeline

pytestmark = pytest.mark.gpu


def _run(pipe, case, ctx, timing, slots=2):
    pipe.set_stage_timing(timing)
    stages = []
    for k, s in enumerate(case["scans"]):
        pipe.stage_scan(k % slots, s)
        pipe.run_scan(k % slots, s, k)
        if timing:
            stages.append(pipe.stage_ms())
    ctx.sync()
    b = pipe.get_beliefs()
    return (b["L"], b["h"], b["X_anchor"], pipe.combined()["L"], pipe.get_iw()["Psi_meas"], pipe.get_map()["map"]), stages


def test_stage_timing_is_bit_neutral_and_consistent(ctx):
    case = cases.build(H=8, n_az=1024, n_scans=3, io="computed")
    ref, _ = _run(_pipeline(case, ctx, 8, case["n"], True), case, ctx, False)
    got, stages = _run(_pipeline(case, ctx, 8, case["n"], True), case, ctx, True)
    for a, b in zip(ref, got):
        assert np.array_equal(a, b)
    names = ("predict", "bins", "evidence", "combine_local", "exchange", "combine_final", "map_update")
    for st in stages:
        assert all(st[f"{k}_ms"] >= 0.0 for k in names)
        assert st["bins_ms"] > 0.0 and st["predict_ms"] > 0.0 and st["evidence_ms"] > 0.0
        parts = sum(st[f"{k}_ms"] for k in names)
        assert abs(parts - st["total_ms"]) <= 1e-3 + 1e-4 * st["total_ms"], st
    from gcslam.diagnostics import tape_from_pipeline, tape_timing_ms
    pipe = _pipeline(case, ctx, 8, case["n"], True)
    pipe.set_stage_timing(True)
    s = case["scans"][0]
    pipe.stage_scan(0, s)
    pipe.run_scan(0, s, 0)
    tm = tape_timing_ms(pipe.stage_ms())
    tape = tape_from_pipeline(pipe, 0, s["scan_end"], s["dt_sec"], s["points"].shape[0], case["n"], timing_ms=tm)
    assert tape.t_total_ms > 0.0 and tape.t_deskew_ms > 0.0 and tape.t_imu_preint_scan_ms > 0.0
    assert tape.t_total_ms >= tape.t_deskew_ms + tape.t_imu_preint_scan_ms
    with pytest.raises(ValueError, match="stage timing"):
        _pipeline(case, ctx, 8, case["n"], True).stage_ms()


def test_host_stats_and_device_runtime_cert(ctx):
    case = cases.build(H=4, n_az=512, n_scans=3, io="computed")
    pipe = _pipeline(case, ctx, 4, case["n"], True)
    pipe.host_stats(reset=True)
    n, M = case["n"], pipe.M
    for k, s in enumerate(case["scans"]):
        pipe.stage_scan(k % 3, s)
        pipe.run_scan(k % 3, s, k)
    ctx.sync()
    h = pipe.host_stats()
    assert h["scans"] == 3 and h["stages"] == 6  # stage_scan + stage_odom per scan
    assert h["h2d_bytes"] == 3 * (8 * (5 * n + 7 * M) + 8 * 84)
    assert h["d2h_bytes"] == 0 and h["jit_recompiles"] == 0
    assert 0.0 < h["scan_enqueue_ms"] and h["scan_enqueue_max_ms"] <= h["scan_enqueue_ms"]
    assert h["scan_wait_ms"] >= 0.0 and h["stage_work_ms"] > 0.0
    b = pipe.get_beliefs()
    cert = pipe.device_runtime_cert()  # consumes
    assert cert.device_to_host_bytes_est == 8 * (4 * (6 + 22 + 484 + 22 + 1))
    assert cert.host_to_device_bytes_est == h["h2d_bytes"]
    assert cert.host_sync_count_est >= 5  # the five getter syncs at least
    assert cert.jit_recompile_count == 0
    assert set(cert.to_dict()) == {"host_sync_count_est", "device_to_host_bytes_est", "host_to_device_bytes_est",
                                   "jit_recompile_count"}
    again = pipe.device_runtime_cert()
    assert again.host_to_device_bytes_est == 0 and again.device_to_host_bytes_est == 0
    assert np.isfinite(b["L"]).all()


def test_conditioning_getters_allocate_nothing_per_call(ctx):
    """The conditioning getters use the pipeline's workspace: repeated calls agree bit for bit and
    leave the host accounting at one sync per download."""
    case = cases.build(H=4, n_az=512, n_scans=1, io="computed")
    pipe = _pipeline(case, ctx, 4, case["n"], True)
    s = case["scans"][0]
    pipe.stage_scan(0, s)
    pipe.run_scan(0, s, 0)
    a, c1 = pipe.hyp_conditioning(), pipe.combined()
    b, c2 = pipe.hyp_conditioning(), pipe.combined()
    assert np.array_equal(a, b) and c1["eig_min"] == c2["eig_min"]


def test_inscan_certs_agree_with_on_demand_jacobi(ctx):
    """The in-scan certificates (Householder + Sturm multisection) against the on-demand Jacobi
    projection of the same stored matrices: eigenvalue extremes at eigh's accuracy, counts exact; the
    scan's other results bit-identical with the certificates on or off."""
    case = cases.build(H=8, n_az=1024, n_scans=2, io="computed")
    outs = []
    for on in (False, True):
        pipe = _pipeline(case, ctx, 8, case["n"], True)
        pipe.set_inscan_certs(on)
        conds = []
        for k, s in enumerate(case["scans"]):
            pipe.stage_scan(0, s)
            pipe.run_scan(0, s, k)
            conds.append(pipe.hyp_conditioning())
        b = pipe.get_beliefs()
        outs.append((conds, b["L"], b["X_anchor"], pipe.combined()["L"]))
    for a, b in zip(outs[0][1:], outs[1][1:]):
        assert np.array_equal(a, b)
    for k, (ref, got) in enumerate(zip(outs[0][0], outs[1][0])):
        np.testing.assert_allclose(got[..., 1], ref[..., 1], rtol=1e-10, atol=0, err_msg=f"scan{k} eig_max")
        assert np.all(np.abs(got[..., 0] - ref[..., 0]) <= 1e-12 * ref[..., 1]), f"scan{k} eig_min"
        np.testing.assert_array_equal(got[..., 3], ref[..., 3], err_msg=f"scan{k} near-null count")
        np.testing.assert_allclose(got[..., 2], got[..., 1] / got[..., 0], rtol=1e-15)
