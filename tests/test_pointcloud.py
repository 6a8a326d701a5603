"""PointCloud2 parsing: parse_pointcloud2_vlp16 (backend_node.py:377-468) and
the no-TF base transform (:1677-1690).

The reference holds no test or fixture for this function, so parity here is pinned only by the
oracle's restatement (the same structured-dtype NumPy read as the reference) — "parity unpinned"
against reference outputs. CPU tests check the oracle's round trip on synthetic messages; GPU
tests compare the device parse with the oracle bit-exactly for ring/tag/times and within
1e-15 relative for points and weights (R p + t summation order, ocml vs libm exp)."""

import numpy as np
import pytest

from oracle import gc_oracle as O

LAYOUTS = [("vlp16", "relative"), ("vlp16", "ns"), ("vlp16", "none"), ("f64", "relative"), ("f64", "none")]


def _scan(n_az=64):
    from gcslam.synth import make_scan
    return make_scan(3, n_az=n_az)


def _oracle(msg, R, t):
    fields = [(f.name, f.offset, f.datatype) for f in msg.fields]
    stamp = msg.header.stamp.sec + msg.header.stamp.nanosec * 1e-9
    p, ts, w, ring, tag = O.parse_pointcloud2_vlp16(msg.data, fields, msg.point_step, msg.width * msg.height, stamp)
    return O.to_base(p, R, t), ts, w, ring, tag


@pytest.mark.parametrize("layout,time_mode", LAYOUTS)
def test_oracle_roundtrip(layout, time_mode):
    from gcslam.synth import make_pointcloud2
    from gcslam.constants import T_BASE_LIDAR
    s = _scan()
    msg = make_pointcloud2(s, layout=layout, time_mode=time_mode)
    R, t = O.T_base_sensor(T_BASE_LIDAR)
    p, ts, w, ring, tag = _oracle(msg, R, t)
    tol = 1e-5 if layout == "vlp16" else 1e-12  # f32 wire coordinates
    assert np.max(np.abs(p - s["points"])) < tol
    assert np.array_equal(ring, s["ring"]) and not tag.any()
    if time_mode == "none":
        assert np.all(ts == msg.header.stamp.sec + msg.header.stamp.nanosec * 1e-9)
    elif time_mode == "ns":
        assert np.max(np.abs(ts - s["timestamps"])) < 1e-9
    else:
        assert np.max(np.abs(ts - (s["timestamps"] - s["scan_start"]))) < 1e-6
    assert np.all((w > 0) & (w <= 1.0))


def test_oracle_nonfinite_and_missing_fields():
    from gcslam.synth import make_pointcloud2
    msg = make_pointcloud2(_scan(), layout="f64", n_nonfinite=9)
    fields = [(f.name, f.offset, f.datatype) for f in msg.fields]
    p, _, w, _, _ = O.parse_pointcloud2_vlp16(msg.data, fields, msg.point_step, msg.width, 0.0)
    big = np.abs(p) == O.NONFINITE_SENTINEL
    assert big.sum() == 9 and np.isfinite(p).all() and np.isfinite(w).all()
    with pytest.raises(RuntimeError):
        O.parse_pointcloud2_vlp16(msg.data, [f for f in fields if f[0] != "ring"], msg.point_step, msg.width, 0.0)
    assert O.parse_pointcloud2_vlp16(b"", fields, msg.point_step, 0, 0.0)[0].shape == (0, 3)


@pytest.mark.gpu
@pytest.mark.parametrize("layout,time_mode", LAYOUTS)
def test_gpu_parse_matches_oracle(ctx, layout, time_mode):
    from gcslam.ops import parse_pointcloud2_vlp16
    from gcslam.synth import make_pointcloud2
    from gcslam.constants import T_BASE_LIDAR
    msg = make_pointcloud2(_scan(256), layout=layout, time_mode=time_mode, n_nonfinite=7)
    R, t = O.T_base_sensor(T_BASE_LIDAR)
    p, ts, w, ring, tag = parse_pointcloud2_vlp16(msg, R, t, ctx=ctx)
    rp, rts, rw, rring, rtag = _oracle(msg, R, t)
    assert np.array_equal(ring, rring) and np.array_equal(tag, rtag)   # integer contract: bit-exact
    assert np.array_equal(ts, rts)                                      # f32/f64 -> f64, x1e-9: exact
    assert np.max(np.abs(p - rp) / np.maximum(np.abs(rp), 1.0)) < 1e-15
    assert np.max(np.abs(w - rw) / rw) < 1e-14


@pytest.mark.gpu
def test_gpu_parse_empty_and_errors(ctx):
    from gcslam.ops import parse_pointcloud2_vlp16
    from gcslam.ops.pointcloud import PointCloud2Msg, PointField
    from gcslam.synth import make_pointcloud2
    empty = PointCloud2Msg(width=0, height=1, point_step=22, fields=[], data=b"")
    assert parse_pointcloud2_vlp16(empty, ctx=ctx)[0].shape == (0, 3)
    msg = make_pointcloud2(_scan())
    msg.fields = [f for f in msg.fields if f.name != "ring"]
    with pytest.raises(RuntimeError):
        parse_pointcloud2_vlp16(msg, ctx=ctx)
    msg = make_pointcloud2(_scan())
    msg.fields = [PointField(f.name, f.offset + (30 if f.name == "x" else 0), f.datatype) for f in msg.fields]
    with pytest.raises(ValueError):
        parse_pointcloud2_vlp16(msg, ctx=ctx)  # field outside point_step: the C entry rejects it


@pytest.mark.gpu
def test_gpu_pipeline_staged_from_pointcloud2(ctx):
    """A scan staged from its PointCloud2 bytes gives the same bin statistics as the same scan
    staged from the (oracle-)parsed arrays: the device parse feeds a1 directly."""
    from gcslam.pipeline import BatchedScanPipeline, PipelineConfig
    from gcslam.synth import make_hypotheses, make_pointcloud2
    from gcslam.constants import T_BASE_LIDAR
    from oracle import cases
    s = _scan(256)
    msg = make_pointcloud2(s, layout="vlp16", time_mode="ns")
    R, t = O.T_base_sensor(T_BASE_LIDAR)
    rp, rts, rw, _, _ = _oracle(msg, R, t)
    n = rp.shape[0]
    out = []
    for mode in ("arrays", "pointcloud2"):
        pipe = BatchedScanPipeline(3, n, PipelineConfig(n_points_cap=n), ctx=ctx)
        hy = make_hypotheses(3)
        pipe.set_beliefs(hy["X_anchor"], hy["z_lin"], hy["L"], hy["h"], hy["stamp"])
        pipe.set_io_mode(True)
        case = cases.build(H=3, n_az=256, n_scans=1)
        pipe.set_iw(*case["iw"])
        pipe.set_map(case["map_record"])
        if mode == "arrays":
            pipe.stage_scan(0, dict(s, points=rp, timestamps=rts, weights=rw))
        else:
            pipe.stage_pointcloud2(0, msg, s, R, t)
        pipe.run_scan(0, s, 0)
        ctx.sync()
        out.append(pipe.bin_stats()[0])
    assert np.max(np.abs(out[0] - out[1]) / np.maximum(np.abs(out[1]), 1e-300)) < 1e-12


def test_imu_window_padded_slicing():
    """backend_node.py:1927-1951: window [min(t_last, start) - 1e-9, max(t_scan, end) + 1e-9], last M
    samples, zero padding."""
    from gcslam.ops import imu_window_padded
    buf = [(0.005 * k, (k, 0.0, 1.0), (0.0, k, 9.81)) for k in range(400)]
    st, gy, ac = imu_window_padded(buf, t_last_scan=0.5, scan_start_time=0.6, t_scan=0.7, scan_end_time=0.65, M=512)
    sel = [t for (t, _, _) in buf if 0.5 - 1e-9 <= t <= 0.7 + 1e-9]
    assert np.count_nonzero(st) == len(sel) and np.allclose(st[:len(sel)], sel)
    assert np.all(st[len(sel):] == 0.0) and np.all(gy[len(sel):] == 0.0)
    assert gy[0, 0] == 100 and ac[0, 1] == 100
    st, _, _ = imu_window_padded(buf, 0.0, 0.0, 2.0, 2.0, M=64)  # more samples than M: the last 64
    assert st[0] == buf[-64][0] and st[-1] == buf[-1][0]
    st, _, _ = imu_window_padded([], 0.0, 0.0, 1.0, 1.0, M=8)
    assert st.shape == (8,) and not st.any()
