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
