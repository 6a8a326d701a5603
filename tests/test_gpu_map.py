"""C5 map update: primitive_map_fuse (+ transform_gaussian_to_world) on the GPU against the
oracle's sequential scatter-add restatement. Without the world transform the per-slot sums are
formed in the same row order as np.add.at, so the result must be bit-exact; with it, the 3x3
solves differ by ulps (LU in ocml vs LAPACK) and the comparison is relative."""

import numpy as np
import pytest

from oracle import gc_oracle as O

pytestmark = pytest.mark.gpu


def _case(rng, K, M, L=3):
    A = rng.normal(size=(K, 3, 3))
    Lam = A @ np.swapaxes(A, 1, 2) + 0.1 * np.eye(3)
    return dict(slots=rng.integers(-5, M + 5, K), Lambdas=Lam, thetas=rng.normal(size=(K, 3)),
                etas=rng.normal(size=(K, L, 3)), weights=rng.uniform(0, 1, K), resp=rng.uniform(0, 1, K),
                valid=rng.uniform(0, 1, K) > 0.2, colors=rng.uniform(-0.2, 1.2, (K, 3)),
                sources=rng.integers(0, 2, K))


def _tile(rng, M, L=3):
    B = rng.normal(size=(M, 3, 3))
    return dict(Lambdas=B @ np.swapaxes(B, 1, 2), thetas=rng.normal(size=(M, 3)), etas=rng.normal(size=(M, L, 3)),
                weights=rng.uniform(0, 2, M), timestamps=rng.uniform(0, 5, M),
                last_supported_scan_seq=rng.integers(0, 9, M).astype(np.int64),
                last_update_scan_seq=rng.integers(0, 9, M).astype(np.int64), cam_mass=rng.uniform(0, 1, M) * (rng.uniform(0, 1, M) > 0.5),
                lidar_mass=rng.uniform(0, 1, M), rgb_cam_accum=rng.uniform(0, 1, (M, 3)),
                rgb_cam_denom=rng.uniform(0, 1, M), rgb=np.full((M, 3), 0.5), colors=np.zeros((M, 3)))


@pytest.mark.parametrize("K,M,world,packed", [(5000, 1 << 12, False, True), (5000, 1 << 12, False, False),
                                              (20000, 1 << 16, False, True), (3000, 2000, True, True),
                                              (3000, 2000, True, False), (1, 10, False, True),
                                              (131072, 1 << 20, False, True), (131072, 1 << 20, True, True),
                                              # every slot in every 256-row sort block: ~79 runs per slot
                                              # (past the staged apply's 8-run slice: the chain walk) and
                                              # 256 (past the gathering apply's 64-run slice)
                                              (20000, 100, False, True), (65536, 16, False, False)])
def test_primitive_map_fuse_matches_oracle(ctx, K, M, world, packed):
    """Two fuses in a row: the first onto uploaded colours (not current: every slot's colour is
    recomputed), the second onto the colours the first left (current: only touched slots are
    recomputed); either device layout."""
    from gcslam.primitive_map import DevicePrimitiveMap, fuse_rows
    rng = np.random.default_rng(K + M)
    c, tile = _case(rng, K, M), _tile(rng, M)
    c2 = _case(rng, K, M)
    dm = DevicePrimitiveMap(1, M, ctx=ctx, packed=packed)
    dm.upload(**tile)
    assert not dm.colors_current
    pose = np.array([1.0, -2.0, 0.0, 0.05, -0.02, 0.7]) if world else None
    ref = tile
    for step, cc in enumerate((c, c2)):
        n = fuse_rows(dm, cc["slots"], cc["Lambdas"], cc["thetas"], cc["etas"], cc["weights"], cc["resp"],
                      7.5 + step, 11 + step, cc["valid"], cc["colors"], cc["sources"], world_pose=pose)
        assert dm.colors_current
        Lm, th, et = cc["Lambdas"], cc["thetas"], cc["etas"]
        if world:
            Lm, th, et = O.transform_gaussian_to_world(Lm, th, et, pose)
        ref, nref = O.primitive_map_fuse(ref, cc["slots"], Lm, th, et, cc["weights"], cc["resp"], 7.5 + step,
                                         11 + step, cc["valid"], cc["colors"], cc["sources"])
        assert n == nref
    got = dm.download()
    for k, v in ref.items():
        if world and k in ("Lambdas", "thetas", "etas", "rgb", "colors"):
            np.testing.assert_allclose(got[k], v, rtol=1e-12, atol=1e-12 * np.max(np.abs(v)), err_msg=k)
        else:
            np.testing.assert_array_equal(got[k], v, err_msg=k)


def test_packed_and_field_layouts_round_trip(ctx):
    """upload -> download through the packed record returns every field bit for bit, and the packed
    record keeps the fuse's read-modify-write fields in its first two 128-B lines."""
    import ctypes as C
    from gcslam import _abi
    from gcslam.primitive_map import DevicePrimitiveMap
    rng = np.random.default_rng(3)
    M = 777
    t = _tile(rng, M)
    t.update(valid_mask=(rng.uniform(0, 1, M) > 0.5).astype(np.uint8), created_timestamps=rng.uniform(0, 1, M),
             primitive_ids=rng.integers(0, 1 << 40, M).astype(np.int64))
    for packed in (True, False):
        dm = DevicePrimitiveMap(1, M, ctx=ctx, packed=packed)
        dm.upload(**t)
        got = dm.download()
        for k, v in t.items():
            np.testing.assert_array_equal(got[k], v, err_msg=k)
    off = np.zeros(16, np.int64)
    sb = C.c_int64(0)
    _abi.call("gc_primitive_map_record_layout", 3, off.ctypes.data, C.byref(sb))
    assert sb.value == 384 and max(off[:11]) + 8 <= 256 and off[2] + 72 <= 256


def test_fuse_colour_estimate_stays_within_the_fused_tile(ctx):
    """The reference recomputes the colour estimate over the fused tile only
    (primitive_map.py:1097-1105): an insert into tile 0 leaves its colours at clip(c), and a fuse
    into tile 1 must not replace them by the estimate."""
    from gcslam import primitive_map as PM
    rng = np.random.default_rng(11)
    m_tile, L = 64, 3
    dm = PM.DevicePrimitiveMap(3, m_tile, ctx=ctx)
    K = 8
    cols = rng.uniform(0, 1, (K, 3))
    PM.primitive_map_insert_masked(dm, 0, np.tile(np.eye(3), (K, 1, 1)), np.zeros((K, 3)), np.zeros((K, L, 3)),
                                   rng.uniform(0.1, 1, K), 0.0, np.ones(K, bool), colors_new=cols,
                                   sources_new=np.zeros(K, np.int32))
    before = dm.download_tile(0, "rgb", "colors")
    assert not dm.colors_current
    c = _case(rng, 200, m_tile)
    PM.primitive_map_fuse(dm, 1, c["slots"], c["Lambdas"], c["thetas"], c["etas"], c["weights"], c["resp"], 2.0,
                          3, valid_mask=c["valid"], colors_meas=c["colors"], sources_meas=c["sources"])
    after = dm.download_tile(0, "rgb", "colors")
    for k in ("rgb", "colors"):
        np.testing.assert_array_equal(after[k], before[k], err_msg=k)
    ref = O.empty_tile(m_tile, L)
    ref, _ = O.primitive_map_fuse(ref, c["slots"], c["Lambdas"], c["thetas"], c["etas"], c["weights"], c["resp"],
                                  2.0, 3, c["valid"], c["colors"], c["sources"])
    got = dm.download_tile(1)
    for k in ("Lambdas", "weights", "cam_mass", "rgb", "colors"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def test_primitive_map_fuse_reference_signature(ctx):
    from gcslam.primitive_map import DevicePrimitiveMap, primitive_map_fuse
    rng = np.random.default_rng(7)
    m_tile = 512
    dm = DevicePrimitiveMap(4, m_tile, ctx=ctx)
    c = _case(rng, 700, m_tile)
    res, cert, eff = primitive_map_fuse(dm, 2, c["slots"], c["Lambdas"], c["thetas"], c["etas"], c["weights"],
                                        c["resp"], 3.0, 5, valid_mask=c["valid"])
    got = dm.download("weights", "timestamps")
    keep = (c["slots"] >= 0) & (c["slots"] < m_tile)
    touched = np.unique(2 * m_tile + c["slots"][keep])
    assert res.n_fused == touched.shape[0] and eff.realized == touched.shape[0] and cert.exact
    assert np.all(got["timestamps"][touched] == 3.0)
    others = np.setdiff1d(np.arange(4 * m_tile), touched)
    assert np.all(got["weights"][others] == 0.0) and np.all(got["timestamps"][others] == 0.0)
    res0, _, _ = primitive_map_fuse(dm, 0, np.zeros(0, np.int64), np.zeros((0, 3, 3)), np.zeros((0, 3)),
                                    np.zeros((0, 3, 3)), np.zeros(0), np.zeros(0), 1.0)
    assert res0.n_fused == 0
