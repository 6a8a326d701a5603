"""PointCloud2 (VLP-16 layout) parsing on the GPU: parse_pointcloud2_vlp16
(backend/backend_node.py:377-468) and the no-TF base transform (backend_node.py:1677-1690); the
IMU window slicing/padding of the same per-scan staging (backend_node.py:1927-1951).

The message is duck-typed like sensor_msgs/PointCloud2: ``width``, ``height``, ``point_step``,
``fields`` (objects with ``name``, ``offset``, ``datatype``), ``data`` (bytes) and
``header.stamp.sec`` / ``header.stamp.nanosec``. ``PointField`` / ``PointCloud2Msg`` below are
minimal stand-ins for callers without ROS message classes. All per-point arithmetic runs in
``gc_pointcloud2_parse``; the host only resolves the field table.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Tuple

import numpy as np

from .. import _abi
from ..constants import GC_MAX_IMU_PREINT_LEN

INT8, UINT8, INT16, UINT16, INT32, UINT32, FLOAT32, FLOAT64 = range(1, 9)


@dataclass
class PointField:
    name: str
    offset: int
    datatype: int
    count: int = 1


@dataclass
class _Stamp:
    sec: int = 0
    nanosec: int = 0


@dataclass
class _Header:
    stamp: _Stamp = field(default_factory=_Stamp)
    frame_id: str = "velodyne"


@dataclass
class PointCloud2Msg:
    width: int
    height: int
    point_step: int
    fields: List[PointField]
    data: bytes
    header: _Header = field(default_factory=_Header)
    is_bigendian: bool = False


def header_stamp_sec(msg) -> float:
    return msg.header.stamp.sec + msg.header.stamp.nanosec * 1e-9


def field_table(msg) -> np.ndarray:
    """int32[10] = [x_off, x_type, y_off, y_type, z_off, z_type, ring_off, ring_type, time_off,
    time_type] (time_off = -1 without a t/time field), the layout of gc_pointcloud2_parse.
    Raises RuntimeError when a VLP-16 field is missing (backend_node.py:396-403)."""
    fmap = {f.name: (int(f.offset), int(f.datatype)) for f in msg.fields}
    missing = [k for k in ("x", "y", "z", "ring") if k not in fmap]
    if missing:
        raise RuntimeError(f"PointCloud2 (VLP-16 layout) missing required fields: {missing}. "
                           f"Present fields: {sorted(fmap)}")
    for k, (_, dt) in fmap.items():
        if not 1 <= dt <= 8:
            raise ValueError(f"Unsupported PointField datatype: {dt}")
    tf = "t" if "t" in fmap else ("time" if "time" in fmap else None)
    t_off, t_type = fmap[tf] if tf else (-1, 0)
    return np.array([*fmap["x"], *fmap["y"], *fmap["z"], *fmap["ring"], t_off, t_type], dtype=np.int32)


def parse_pointcloud2_vlp16(msg, R_base_lidar=None, t_base_lidar=None, ctx=None
                            ) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """(points, timestamps, weights, ring, tag) as the reference returns them; with an extrinsic
    (R_base_lidar (3,3), t_base_lidar (3,)) the points come out in the base frame."""
    ctx = ctx or _abi.default_context()
    n = int(msg.width) * int(msg.height)
    if n <= 0:
        return (np.zeros((0, 3)), np.zeros(0), np.zeros(0), np.zeros(0, np.uint8), np.zeros(0, np.uint8))
    ft = field_table(msg)
    step = int(msg.point_step)
    raw = np.frombuffer(bytes(msg.data), dtype=np.uint8, count=n * step)
    R = np.eye(3) if R_base_lidar is None else np.ascontiguousarray(R_base_lidar, np.float64).reshape(3, 3)
    t = np.zeros(3) if t_base_lidar is None else np.ascontiguousarray(t_base_lidar, np.float64).reshape(3)
    d_raw = _abi.DeviceArray.from_host(ctx, raw, np.uint8)
    pts, ts, ws = _abi.DeviceArray(ctx, (n, 3)), _abi.DeviceArray(ctx, n), _abi.DeviceArray(ctx, n)
    rg, tg = _abi.DeviceArray(ctx, n, np.uint8), _abi.DeviceArray(ctx, n, np.uint8)
    Ra, Rp = _abi.f64p(R)  # keep the host arrays alive across the call
    ta, tp = _abi.f64p(t)
    _abi.call("gc_pointcloud2_parse", ctx.handle, d_raw.ptr, n, step, ft.ctypes.data, header_stamp_sec(msg), Rp, tp,
              pts.ptr, ts.ptr, ws.ptr, rg.ptr, tg.ptr, ctx=ctx)
    return pts.download(), ts.download(), ws.download(), rg.download(), tg.download()


def imu_message_to_base(gyro, accel, R_base_imu, accel_scale: float = 1.0) -> Tuple[np.ndarray, np.ndarray]:
    """The node's IMU callback transform (on_imu, backend_node.py:1397-1412): accel · imu_accel_scale,
    then gyro_base = R_base_imu @ gyro and accel_base = R_base_imu @ accel. One message's 3-vectors (or
    (n, 3) rows of several). The reference keeps this callback CPU-only by design (no device work per
    message, :1400); the rotated samples feed imu_window_padded."""
    R = np.asarray(R_base_imu, np.float64).reshape(3, 3)
    g = np.asarray(gyro, np.float64)
    a = np.asarray(accel, np.float64) * float(accel_scale)
    if g.ndim == 1:
        return R @ g, R @ a
    return np.einsum("ij,nj->ni", R, g), np.einsum("ij,nj->ni", R, a)


def imu_window_padded(imu_buffer, t_last_scan: float, scan_start_time: float, t_scan: float,
                      scan_end_time: float, M: int = GC_MAX_IMU_PREINT_LEN
                      ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """The node's IMU slicing and padding (backend_node.py:1927-1951): samples (t, gyro, accel)
    with t in [min(t_last_scan, scan_start) - 1e-9, max(t_scan, scan_end) + 1e-9], the last M of
    them, zero-padded to M rows -> (stamps (M,), gyro (M, 3), accel (M, 3)), the arrays
    stage_pointcloud2 / stage_scan take as imu_stamps / imu_gyro / imu_accel. Host bookkeeping
    over the node's Python ring buffer (no arithmetic to offload)."""
    t_min = min(t_last_scan, scan_start_time)
    t_max = max(t_scan, scan_end_time)
    eps_t = 1e-9
    window = [(t, g, a) for (t, g, a) in imu_buffer if t_min - eps_t <= t <= t_max + eps_t]
    if len(window) > M:
        window = window[-M:]
    stamps, gyro, accel = np.zeros(M), np.zeros((M, 3)), np.zeros((M, 3))
    for i, (t, g, a) in enumerate(window):
        stamps[i] = float(t)
        gyro[i] = np.asarray(g, np.float64)
        accel[i] = np.asarray(a, np.float64)
    return stamps, gyro, accel
