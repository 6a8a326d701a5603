"""The hot path on the reference's own sensor data (docs/raw_sensor_dump via tests/golden/raw_sensor.npz):
3,000 real IMU samples (~203 Hz, base frame through the dump's extrinsic and the 9.81 g -> m/s² scale,
backend_node.py:1397-1412) and 300 real odometry messages (first-odom-as-origin, :1512-1514), cut
into consecutive 0.1 s scan windows exactly as the node cuts them (the IMU window of
backend_node.py:1927-1951, zero-padded to 512; the odometry sample closest to the scan stamp,
:1805-1815; t_last / dt_sec of :1788-1822, the first scan with its empty scan-to-scan interval).
Stamps stay absolute (~1.73e9 s), as the node passes them. The points stay synthetic (re-timed into
each sweep); the dump holds no covariances (SURVEY §8d's are used, with the node's z cap).

  * the IMU soft windows and the weighted preintegration (a3) on every real window;
  * the IMU/odom evidence branch computed on the device (pipeline.py:595-776) over 24 consecutive
    scans at H = 4, against the oracle pipeline run alongside (chained, no re-seeding);
  * the full batched pipeline at the C3 bars (test_gpu_configs._run_and_compare: each scan re-seeded
    from the device state) at H = 4 over 24 scans and at H = 256 x 65,536 points over 3 scans.
"""

import numpy as np
import pytest

from oracle import cases
from oracle import gc_oracle as O
from test_gpu_configs import _run_and_compare

pytestmark = pytest.mark.gpu

N_SCANS = 24


def _rel(a, b, floor=1e-300):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), floor))


def test_preintegration_on_real_imu_windows(ctx):
    from gcslam.ops import smooth_window_weights
    from gcslam.ops.imu_preintegration import preintegrate_imu_batch
    st = cases.raw_sensor_streams()
    t0 = float(st["imu_stamps"][0]) + 0.05
    rng = np.random.default_rng(61)
    H = 3
    r0 = rng.normal(0, 0.2, (H, 3)); bg = rng.normal(0, 1e-3, (H, 3)); ba = rng.normal(0, 1e-2, (H, 3))
    for k in range(N_SCANS):
        s = cases.raw_sensor_scan(st, k, t0, first=(k == 0))
        t, g, a = s["imu_stamps"], s["imu_gyro"], s["imu_accel"]
        for lo, hi, sig in ((s["scan_start"], s["scan_end"], 0.01), (s["t_last"], s["t_scan"], 0.02)):
            w = smooth_window_weights(t, lo, hi, sig, ctx=ctx)
            np.testing.assert_allclose(w, O.smooth_window_weights(t, lo, hi, sig), rtol=1e-13, atol=1e-300)
        out = preintegrate_imu_batch(t, g, a, w, r0, bg, ba, ctx=ctx)
        for h in range(H):
            ref = O.preintegrate(t, g, a, w, r0[h], bg[h], ba[h])
            tag = f"window {k} hyp {h}"
            assert np.max(np.abs(out[h, 0:6] - ref["delta_pose"])) < 1e-11, tag
            assert np.max(np.abs(out[h, 6:15].reshape(3, 3) - ref["delta_R"])) < 1e-13, tag
            assert _rel(out[h, 18:21], ref["delta_v"]) < 1e-11, tag
            assert abs(out[h, 21] - ref["ess"]) < 1e-12 * ref["ess"], tag
            for j, key in ((22, "a_body_mean"), (25, "a_world_nog_mean"), (28, "a_world_mean")):
                assert _rel(out[h, j:j + 3], ref[key]) < 1e-11, (tag, key)
            assert abs(out[h, 31] - ref["dt_eff_sum"]) < 1e-13, tag
        dt_int = O.imu_integration_time(t, s["t_last"], s["t_scan"])
        assert (dt_int == 0.0) if k == 0 else (0.08 < dt_int <= 0.1), (k, dt_int)  # the first scan's interval is empty


def test_io_branch_on_real_sensor_windows(ctx):
    """H = 4, 24 consecutive real windows (the first the node's first scan), 4,096-point synthetic
    sweeps: L_io / h_io / certs / factor parts and the final beliefs against the oracle pipeline
    chained alongside (the iobranch test's bars)."""
    from gcslam.pipeline import BatchedScanPipeline, PipelineConfig
    H = 4
    case = cases.build_raw_sensor(H=H, n_az=256, n_scans=N_SCANS, k0=0)
    pipe = BatchedScanPipeline(H, case["n"], PipelineConfig(n_points_cap=case["n"]), ctx=ctx)
    hy = case["hyp"]
    pipe.set_beliefs(hy["X_anchor"], hy["z_lin"], hy["L"], hy["h"], hy["stamp"])
    pipe.set_weights(hy["weights"])
    pipe.set_io_mode(True)
    pipe.set_iw(*case["iw"])
    pipe.set_map(case["map_record"])
    st = case["state"]
    for k, s in enumerate(case["scans"]):
        pipe.stage_scan(0, s)
        pipe.run_scan(0, s, st.scan_count)
        st, comb, res = O.process_scan(st, cases.scan_input(s), None, case["bins"], case["cfg"])
        ctx.sync()
        L, h, cert = pipe.io_evidence()
        parts = pipe.io_parts()
        bel = pipe.get_beliefs()
        diag = pipe.hyp_diag()
        for i in range(H):
            io, p = res[i]["io"], res[i]["io_parts"]
            tag = (k, i)
            assert _rel(L[i], io.L) < 1e-9, (tag, _rel(L[i], io.L))
            assert _rel(h[i], io.h) < 1e-8, (tag, _rel(h[i], io.h))
            assert abs(cert[i, 9] - io.trig) <= 1e-9 * max(1.0, io.trig), (tag, cert[i, 9], io.trig)
            assert abs(cert[i, 8] - io.nll) <= 1e-8 * max(1.0, abs(io.nll)), (tag, cert[i, 8], io.nll)
            assert abs(cert[i, 1] - io.ess[1]) <= 1e-12 * max(1.0, io.ess[1]), tag
            assert abs(cert[i, 4] - io.support[1]) <= 1e-12, tag
            assert _rel(parts[i, 0:6], p["odom"]["delta_z"][0:6]) < 1e-9, tag
            assert _rel(parts[i, 13:16], p["gyro"]["r_rot"]) < 1e-8, tag
            assert _rel(parts[i, 16:19], p["preint"]["r_vel"]) < 1e-8, tag
            assert _rel(parts[i, 28:31], p["kinematic"]["r_trans"]) < 1e-9, tag
            assert abs(parts[i, 38] - O.imu_integration_time(s["imu_stamps"], s["t_last"], s["t_scan"])) < 1e-12, tag
            b = res[i]["belief"]
            assert np.max(np.abs(diag[i, 0:6] - res[i]["pose"])) < 1e-6, tag           # north-star bar
            assert np.max(np.abs(bel["X_anchor"][i] - b.X_anchor)) < 1e-6, tag
            assert _rel(bel["L"][i], b.L) < 1e-8, tag
        c = pipe.combined()
        assert _rel(c["L"], comb["L"]) < 1e-8, k
    pipe.close()


def test_pipeline_on_real_sensor_windows_h4(ctx):
    """H = 4 over 24 consecutive real windows, 16,384-point sweeps, every hypothesis at the C3 bars."""
    case = cases.build_raw_sensor(H=4, n_az=1024, n_scans=N_SCANS, k0=0)
    pipe = _run_and_compare(ctx, case, 4, case["n"], [0, 1, 2, 3], N_SCANS, True)
    pipe.close()


def test_pipeline_on_real_sensor_windows_c3(ctx):
    """C3 geometry (65,536 points x 256 hypotheses) over 3 consecutive real windows, sampled hypotheses
    at the C3 bars (all-hypothesis coupling checked through the combine / IW / map)."""
    case = cases.build_raw_sensor(H=256, n_az=4096, n_scans=3, k0=5)
    pipe = _run_and_compare(ctx, case, 256, case["n"], [0, 1, 127, 255], 3, True)
    pipe.close()
