"""TEST INFRASTRUCTURE — builds identical inputs for the oracle and the GPU pipeline
(synthetic scans, hypotheses, IMU/odom evidence, IW priors, warm-up map)."""

from __future__ import annotations

import numpy as np

from . import gc_oracle as O

SCAN_KEYS = ["points", "timestamps", "weights", "ring", "tag", "imu_stamps", "imu_gyro", "imu_accel",
             "scan_start", "scan_end", "t_last", "t_scan", "dt_sec"]


def scan_input(s):
    odom = (O.OdomInput(s["odom_pose"], s["odom_cov"], s["odom_twist"], s["odom_twist_cov"])
            if "odom_pose" in s else None)
    return O.ScanInput(**{k: s[k] for k in SCAN_KEYS}, odom=odom)


def warmup_map(scan, cap, origin, bins, yaw0=0.0):
    """MapBinStats of one warm-up scan placed at the pose Rz(yaw0) (no deskew, zero pose cov)."""
    bud = O.point_budget_resample(scan["points"], scan["timestamps"], scan["weights"], None, None, cap)
    sa = O.bin_soft_assign(O.point_directions(bud["points"], origin), bins)
    mm = O.scan_bin_moment_match(bud["points"], None, bud["weights"], sa["resp"], None, origin)
    return O.pose_cov_inflation_pushforward(mm, O.so3_exp(np.array([0.0, 0.0, yaw0])), np.zeros(3), np.zeros((6, 6)))


def turn_world(scan, yaw0):
    """The same scan seen by a robot whose world (and odometry) frame starts rotated by yaw0:
    the odometry pose becomes Rz(yaw0) ∘ pose (body-frame twists, points and IMU unchanged)."""
    s = dict(scan)
    if "odom_pose" in s:
        s["odom_pose"] = O.se3_compose(np.array([0.0, 0.0, 0.0, 0.0, 0.0, yaw0]), s["odom_pose"])
    return s


def map_to_record(m: O.MapStats):
    B = m.N_dir.shape[0]
    return np.concatenate([m.S_dir, m.S_dir_scatter.reshape(B, 9), m.N_dir[:, None], m.N_pos[:, None],
                           m.sum_p, m.sum_ppT.reshape(B, 9)], axis=1)


RAW_SENSOR_NPZ = "tests/golden/raw_sensor.npz"  # tests/golden/make_raw_sensor.py (the reference's sensor dump)
RAW_SCAN_PERIOD = 0.1


def imu_window(stamps, gyro, accel, t_last_scan, scan_start_time, t_scan, scan_end_time, M=512):
    """The node's IMU slicing and padding (backend_node.py:1927-1951) over a time-ordered buffer:
    samples with t in [min(t_last, scan_start) - 1e-9, max(t_scan, scan_end) + 1e-9], the last M of
    them, zero-padded to M rows."""
    t_min, t_max = min(t_last_scan, scan_start_time), max(t_scan, scan_end_time)
    sel = np.nonzero((stamps >= t_min - 1e-9) & (stamps <= t_max + 1e-9))[0][-M:]
    st, gy, ac = np.zeros(M), np.zeros((M, 3)), np.zeros((M, 3))
    st[:sel.shape[0]], gy[:sel.shape[0]], ac[:sel.shape[0]] = stamps[sel], gyro[sel], accel[sel]
    return st, gy, ac


def raw_sensor_streams(root=None):
    """The reference's raw sensor dump as the node receives it: the 3,000 IMU samples in the base
    frame (on_imu, backend_node.py:1397-1412, with the dump's extrinsic and the 9.81 g -> m/s² scale)
    and the 300 odometry messages relative to the first one (on_odom, :1441-1540). The dump holds no
    covariances: the pose covariance is SURVEY §8d's diag(1e-2 x3, 1e-3 x3) with the node's z cap
    (1e6) and the twist covariance 1e-2·I."""
    import os
    root = root or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    g = np.load(os.path.join(root, RAW_SENSOR_NPZ))
    imu = g["imu_raw_3000"]
    R, _ = O.T_base_sensor(O.DUMP_T_BASE_IMU)
    gyro, accel = O.imu_to_base(imu[:, 1:4], imu[:, 4:7], R, O.DUMP_ACCEL_SCALE)
    od = g["odom_300"]
    absp = [O.odom_pose_from_msg(r[1:4], r[4:8]) for r in od]
    rel = np.stack([O.odom_relative(absp[0], p) for p in absp])
    cov = O.odom_cov_capped(np.diag([1e-2, 1e-2, 1e-2, 1e-3, 1e-3, 1e-3]))
    return dict(imu_stamps=imu[:, 0].copy(), imu_gyro=gyro, imu_accel=accel, odom_stamps=od[:, 0].copy(),
                odom_pose=rel, odom_twist=od[:, 8:14].copy(), odom_cov=cov, odom_twist_cov=1e-2 * np.eye(6))


def raw_sensor_scan(streams, k, t0, first=False, base=None):
    """Scan k of the real-data timeline: the sweep [t0 + 0.1 k, t0 + 0.1 (k + 1)], header stamp =
    sweep end (t_scan), t_last = the previous scan's stamp (the first scan: t_last = t_scan, its
    scan-to-scan interval empty, backend_node.py:1822), dt_sec = sqrt(dt_raw² + eps) (:1788-1794);
    the IMU window of the node (:1927-1951) and the odometry sample closest to t_scan (:1805-1815).
    base: a synthetic scan (gcslam.synth.make_scan) whose points are re-timed into the sweep."""
    T0 = t0 + RAW_SCAN_PERIOD * k
    t_scan = T0 + RAW_SCAN_PERIOD
    s = dict(base) if base is not None else {}
    if base is not None:
        s["timestamps"] = base["timestamps"] - base["scan_start"] + T0
        tmin, tmax = float(np.min(s["timestamps"])), float(np.max(s["timestamps"]))
        scan_start, scan_end = min(t_scan, tmin), max(t_scan, tmax)
    else:
        scan_start, scan_end = T0, t_scan
    t_last = t_scan if first else T0
    dt_raw = (t_scan - t_last) if not first else (scan_end - scan_start)
    st, gy, ac = imu_window(streams["imu_stamps"], streams["imu_gyro"], streams["imu_accel"], t_last, scan_start,
                            t_scan, scan_end)
    j = int(np.argmin(np.abs(streams["odom_stamps"] - t_scan)))
    s.update(imu_stamps=st, imu_gyro=gy, imu_accel=ac, scan_start=scan_start, scan_end=scan_end, t_last=t_last,
             t_scan=t_scan, dt_sec=float(np.sqrt(dt_raw ** 2 + O.F64_EPS)), odom_pose=streams["odom_pose"][j].copy(),
             odom_cov=streams["odom_cov"].copy(), odom_twist=streams["odom_twist"][j].copy(),
             odom_twist_cov=streams["odom_twist_cov"].copy(), odom_index=j)
    return s


def build_raw_sensor(H=4, n_az=256, n_scans=20, k0=1, cap=None):
    """build(io="computed") with the reference's real IMU / odometry (raw_sensor_streams) in place of
    the synthetic IMU and odometry; the points stay synthetic (re-timed into each sweep). Scans k0 ..
    k0 + n_scans - 1 of the timeline that starts 0.05 s after the first IMU sample (k0 = 0: the
    node's first scan, empty scan-to-scan interval)."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fl-slam_amd"))
    from gcslam import synth
    streams = raw_sensor_streams()
    t0 = float(streams["imu_stamps"][0]) + 0.05
    base = [synth.make_scan(k, n_az=n_az) for k in range(n_scans + 1)]
    scans = [raw_sensor_scan(streams, k0 + k, t0, first=(k0 + k == 0), base=base[k + 1]) for k in range(n_scans)]
    n = scans[0]["points"].shape[0] if cap is None else int(cap)
    cfg = O.PipeConfig(n_points_cap=n)
    bins = O.fibonacci_atlas(48)
    hy = synth.make_hypotheses(H)
    Lio, hio, cert = synth.make_io_evidence(H)
    m0 = warmup_map(base[0], n, cfg.lidar_origin, bins)
    nuP, PsiP = O.iw_process_init()
    nuM, PsiM = O.iw_meas_init()
    beliefs = [O.Belief(hy["X_anchor"][i].copy(), hy["z_lin"][i].copy(), hy["L"][i].copy(), hy["h"][i].copy())
               for i in range(H)]
    state = O.ScanState(beliefs, hy["weights"].copy(), nuP, PsiP, nuM, PsiM, m0, 0)
    return dict(scans=scans, n=n, cfg=cfg, bins=bins, hyp=hy, io=(Lio, hio, cert), ios=None, state=state,
                map_record=map_to_record(m0), iw=(nuP, PsiP, nuM, PsiM), streams=streams)


def build(H=4, n_az=256, n_scans=3, seed_scan0=0, io="synthetic", cap=None, yaw0=None, hyp_yaws=None, tilt=0.0):
    """io="synthetic": given IMU/odom-branch evidence (ios list); io="computed": the branch is
    evaluated from each scan's odometry + IMU window (ios=None). cap: N_POINTS_CAP (default: the
    scan size, stride 1). yaw0: the world frame turned by yaw0 (warm-up map and odometry);
    hyp_yaws / tilt: the hypotheses' anchor yaws (cycled) and roll/pitch spread
    (synth.make_hypotheses)."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fl-slam_amd"))
    from gcslam import synth
    scans = [synth.make_scan(seed_scan0 + k, n_az=n_az) for k in range(n_scans + 1)]
    if yaw0 is not None:
        scans = [turn_world(s, yaw0) for s in scans]
    n = scans[0]["points"].shape[0] if cap is None else int(cap)
    cfg = O.PipeConfig(n_points_cap=n)
    bins = O.fibonacci_atlas(48)
    hy = synth.make_hypotheses(H, yaws=hyp_yaws, tilt=tilt)
    Lio, hio, cert = synth.make_io_evidence(H)
    m0 = warmup_map(scans[0], n, cfg.lidar_origin, bins, 0.0 if yaw0 is None else yaw0)
    nuP, PsiP = O.iw_process_init()
    nuM, PsiM = O.iw_meas_init()
    beliefs = [O.Belief(hy["X_anchor"][i].copy(), hy["z_lin"][i].copy(), hy["L"][i].copy(), hy["h"][i].copy())
               for i in range(H)]
    ios = [O.IOEvidence(Lio[i], hio[i], cert[i, 0:3], cert[i, 3:6], cert[i, 6], cert[i, 7], cert[i, 8], cert[i, 9])
           for i in range(H)] if io == "synthetic" else None
    state = O.ScanState(beliefs, hy["weights"].copy(), nuP, PsiP, nuM, PsiM, m0, 0)
    return dict(scans=scans[1:], n=n, cfg=cfg, bins=bins, hyp=hy, io=(Lio, hio, cert), ios=ios, state=state,
                map_record=map_to_record(m0), iw=(nuP, PsiP, nuM, PsiM))
