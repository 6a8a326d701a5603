"""TEST INFRASTRUCTURE — packs the reference's own raw sensor dump into tests/golden/raw_sensor.npz.

The reference ships the only real numeric sensor data of the project under
docs/raw_sensor_dump/ (README.md there: the first IMU / odometry messages of an archived bag):

  imu_raw_first_300.csv, imu_raw_first_3000.csv   stamp, gyro (rad/s), accel (g), IMU frame
  odom_raw_first_300.csv                          stamp, position, quaternion, body twist
  imu_extrinsic_applied_first_300.csv             the reference tool's output for the first 300:
  imu_linear_first_300.csv                        R_base_imu @ (gyro, accel·9.81) [+ gravity_W]
                                                  (tools/apply_imu_extrinsic_to_csv.py:85-110)

The CSVs are data: this script reads them in place (the reference tree exists only in the build
container) and stores the parsed float64 arrays, parsed exactly as the reference tool parses them
(csv.DictReader + float(), apply_imu_extrinsic_to_csv.py:87-101), so the GPU box reads the npz.
Nothing here computes anything: the base-frame transform and the scan windows are the oracle's
(oracle/gc_oracle.py imu_to_base, odom_pose_from_msg; oracle/cases.py build_raw_sensor).

    python tests/golden/make_raw_sensor.py [/root/reference]
"""

from __future__ import annotations

import csv
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
IMU_COLS = ["stamp_sec", "gyro_x", "gyro_y", "gyro_z", "accel_x", "accel_y", "accel_z"]
ODOM_COLS = ["stamp_sec", "x", "y", "z", "qx", "qy", "qz", "qw", "vx", "vy", "vz", "wx", "wy", "wz"]


def _read(path, cols):
    with open(path) as f:
        r = csv.DictReader(f)
        assert list(r.fieldnames) == cols, (path, r.fieldnames)
        return np.array([[float(row[c]) for c in cols] for row in r], dtype=np.float64)


def main(ref_root="/root/reference"):
    d = os.path.join(ref_root, "docs", "raw_sensor_dump")
    out = dict(
        imu_raw_300=_read(os.path.join(d, "imu_raw_first_300.csv"), IMU_COLS),
        imu_raw_3000=_read(os.path.join(d, "imu_raw_first_3000.csv"), IMU_COLS),
        imu_extrinsic_300=_read(os.path.join(d, "imu_extrinsic_applied_first_300.csv"), IMU_COLS),
        imu_linear_300=_read(os.path.join(d, "imu_linear_first_300.csv"), IMU_COLS),
        odom_300=_read(os.path.join(d, "odom_raw_first_300.csv"), ODOM_COLS),
    )
    assert out["imu_raw_300"].shape == (300, 7) and out["imu_raw_3000"].shape == (3000, 7)
    assert np.array_equal(out["imu_raw_3000"][:300], out["imu_raw_300"])
    assert out["odom_300"].shape == (300, 14)
    dst = os.path.join(HERE, "raw_sensor.npz")
    np.savez_compressed(dst, **out)
    print("wrote", dst, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main(*sys.argv[1:])
