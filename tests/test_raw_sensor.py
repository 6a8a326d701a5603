"""The reference's own sensor data (docs/raw_sensor_dump, packed by tests/golden/make_raw_sensor.py)
pins the IMU base-frame transform and the node's per-scan host staging (CPU).

  * tools/apply_imu_extrinsic_to_csv.py:85-110 wrote imu_extrinsic_applied_first_300.csv and
    imu_linear_first_300.csv from imu_raw_first_300.csv with the dump's extrinsic: the oracle's
    T_base_sensor (rotvec -> R, backend_node.py:247-258) and its on_imu restatement (accel · 9.81,
    R @ gyro, R @ accel; backend_node.py:1397-1412) reproduce both files to 1e-12 relative, and so
    does the product's host helper gcslam.ops.imu_message_to_base;
  * the real-data scan windows (oracle/cases.py build_raw_sensor): the product's imu_window_padded
    slices the same samples as the oracle's restatement of backend_node.py:1927-1951, bit for bit;
  * first-odom-as-origin (backend_node.py:1512-1514): first ∘ relative = absolute.
"""

import os

import numpy as np

from oracle import cases
from oracle import gc_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _g():
    return np.load(os.path.join(ROOT, cases.RAW_SENSOR_NPZ))


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


def test_oracle_reproduces_the_reference_extrinsic_csvs():
    g = _g()
    raw, ext, lin = g["imu_raw_300"], g["imu_extrinsic_300"], g["imu_linear_300"]
    R, t = O.T_base_sensor(O.DUMP_T_BASE_IMU)
    assert np.array_equal(t, np.zeros(3))
    gy, ac = O.imu_to_base(raw[:, 1:4], raw[:, 4:7], R, O.DUMP_ACCEL_SCALE)
    assert np.array_equal(ext[:, 0], raw[:, 0]) and np.array_equal(lin[:, 0], raw[:, 0])  # stamps untouched
    assert _rel(gy, ext[:, 1:4]) <= 1e-12, _rel(gy, ext[:, 1:4])
    assert _rel(ac, ext[:, 4:7]) <= 1e-12, _rel(ac, ext[:, 4:7])
    assert _rel(gy, lin[:, 1:4]) <= 1e-12
    assert _rel(ac + O.GRAVITY_W, lin[:, 4:7]) <= 1e-12, _rel(ac + O.GRAVITY_W, lin[:, 4:7])
    # the stationary robot: specific force ≈ +g along base z after the rotation
    assert abs(np.mean(ac[:, 2]) - 9.7) < 0.1


def test_product_imu_transform_matches_the_reference_csvs():
    from gcslam.ops import imu_message_to_base
    g = _g()
    raw, ext = g["imu_raw_300"], g["imu_extrinsic_300"]
    R, _ = O.T_base_sensor(O.DUMP_T_BASE_IMU)
    gy, ac = imu_message_to_base(raw[:, 1:4], raw[:, 4:7], R, O.DUMP_ACCEL_SCALE)
    assert _rel(gy, ext[:, 1:4]) <= 1e-12 and _rel(ac, ext[:, 4:7]) <= 1e-12
    for i in (0, 1, 157, 299):  # one message at a time, as the callback runs
        g1, a1 = imu_message_to_base(raw[i, 1:4], raw[i, 4:7], R, O.DUMP_ACCEL_SCALE)
        assert np.max(np.abs(g1 - ext[i, 1:4])) <= 1e-12 * np.max(np.abs(ext[i, 1:4]))
        assert np.max(np.abs(a1 - ext[i, 4:7])) <= 1e-12 * np.max(np.abs(ext[i, 4:7]))


def test_real_scan_windows_match_the_product_slicer():
    from gcslam.ops import imu_window_padded
    st = cases.raw_sensor_streams()
    buf = list(zip(st["imu_stamps"], st["imu_gyro"], st["imu_accel"]))
    t0 = float(st["imu_stamps"][0]) + 0.05
    counts = []
    for k in range(0, 140):  # 14 s of 0.1 s sweeps, the first with an empty scan-to-scan interval
        s = cases.raw_sensor_scan(st, k, t0, first=(k == 0))
        a = imu_window_padded(buf, s["t_last"], s["scan_start"], s["t_scan"], s["scan_end"])
        for x, y in zip(a, (s["imu_stamps"], s["imu_gyro"], s["imu_accel"])):
            assert np.array_equal(x, y), k
        n = int(np.count_nonzero(s["imu_stamps"]))
        counts.append(n)
        v = s["imu_stamps"][:n]
        assert np.all(np.diff(v) > 0) and v[0] >= min(s["t_last"], s["scan_start"]) - 1e-9
        assert v[-1] <= max(s["t_scan"], s["scan_end"]) + 1e-9
        assert abs(st["odom_stamps"][s["odom_index"]] - s["t_scan"]) <= 0.026  # ~20 Hz odometry
    assert min(counts) >= 19 and max(counts) <= 22, (min(counts), max(counts))  # ~203 Hz IMU


def test_first_odom_as_origin_round_trip():
    g = _g()
    od = g["odom_300"]
    st = cases.raw_sensor_streams()
    first = O.odom_pose_from_msg(od[0, 1:4], od[0, 4:8])
    assert np.max(np.abs(st["odom_pose"][0])) < 1e-12
    for i in (1, 50, 299):
        absp = O.odom_pose_from_msg(od[i, 1:4], od[i, 4:8])
        back = O.se3_compose(first, st["odom_pose"][i])
        assert np.max(np.abs(back - absp)) < 1e-12
    assert st["odom_cov"][2, 2] == O.ODOM_Z_VARIANCE_PRIOR  # backend_node.py:1523 z cap
