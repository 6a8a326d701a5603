"""PrimitiveMap maintenance: insert_masked, cull, forget, recency_inflate and
merge_reduce (backend/structures/primitive_map.py:807-2030).

CPU: the oracle restatement against the reference's own tests for these operators
(test/test_primitive_map_merge_reduce.py:76-99, test/test_map_color_provenance.py:72-87) and the
semantics the reference code defines (eviction order = stable sort on the retention key, ids by
prefix count, max_primitives threshold). GPU: the device operators against the oracle on seeded
tiles: masks, slots, ids and counts bit-exact; float fields within 1e-12 relative (exp / 3x3
LU differ from libm / LAPACK by ulps)."""

import numpy as np
import pytest

from oracle import gc_oracle as O

L = 3


def _eye_tile(m_tile):
    return O.empty_tile(m_tile, L)


def _merge_kat_tile():
    """test_primitive_map_merge_reduce.py:12-73: three unit-precision primitives, two 1 cm apart."""
    t = O.empty_tile(3, L)
    mu = np.array([[0.0, 0.0, 0.0], [0.01, 0.0, 0.0], [10.0, 0.0, 0.0]])
    t["Lambdas"][:] = np.eye(3)
    t["thetas"][:] = mu
    t["weights"][:] = 1.0
    t["primitive_ids"][:] = [0, 1, 2]
    t["valid_mask"][:] = True
    t["cam_mass"][:] = [1.0, 0.0, 0.0]
    t["lidar_mass"][:] = [0.0, 1.0, 1.0]
    t["rgb_cam_accum"][0] = [1.0, 0.0, 0.0]
    t["rgb_cam_denom"][:] = [1.0, 0.0, 0.0]
    t["rgb"][0] = [1.0, 0.0, 0.0]
    return t


def test_oracle_merge_reduce_close_pair_kat():
    out, n = O.primitive_map_merge_reduce(_merge_kat_tile(), merge_threshold=0.5, max_pairs=1)
    assert n == 1
    assert bool(out["valid_mask"][0]) and not bool(out["valid_mask"][1]) and bool(out["valid_mask"][2])
    assert np.isclose(out["weights"][0], 2.0) and out["weights"][1] == 0.0


def _insert_single(tile, color, source, next_id=0):
    return O.primitive_map_insert_masked(tile, np.eye(3)[None], np.zeros((1, 3)), np.zeros((1, L, 3)),
                                         np.array([1.0]), 0.0, np.array([True]), 0, O_RECENCY, next_id,
                                         colors=np.array([color], float), sources=np.array([source]))


def _fuse_single(tile, color, source):
    out, _ = O.primitive_map_fuse(tile, [0], np.eye(3)[None], np.zeros((1, 3)), np.zeros((1, L, 3)), [1.0], [1.0],
                                  1.0, 1, valid=[True], colors=np.array([color], float), sources=np.array([source]))
    return out


O_RECENCY = 0.02


@pytest.mark.parametrize("first,second,expect", [
    (([1.0, 0.0, 0.0], 0), ([0.2, 0.2, 0.2], 1), [1.0, 0.0, 0.0]),   # camera then lidar keeps camera colour
    (([0.2, 0.2, 0.2], 1), ([0.0, 1.0, 0.0], 0), [0.0, 1.0, 0.0]),   # lidar then camera switches to camera
])
def test_oracle_color_provenance_kat(first, second, expect):
    """test_map_color_provenance.py:72-87."""
    t, n, ids, slots = _insert_single(O.empty_tile(1, L), *first)
    assert n == 1 and ids[0] == 0 and slots[0] == 0
    t = _fuse_single(t, *second)
    np.testing.assert_allclose(t["rgb"][0], expect, atol=1e-6)


def test_oracle_insert_slot_order_and_ids():
    t = O.empty_tile(8, L)
    t["valid_mask"][[1, 4]] = True
    t["weights"][[1, 4]] = [0.5, 0.1]
    mask = np.array([True, False, True, True, True, True, True])
    K = mask.shape[0]
    out, n, ids, slots = O.primitive_map_insert_masked(t, np.tile(np.eye(3), (K, 1, 1)), np.ones((K, 3)),
                                                       np.zeros((K, L, 3)), np.full(K, 2.0), 3.0, mask, 5, 0.02, 10)
    # empty slots first in slot order, then valid ones by retention (0.1 < 0.5)
    assert list(slots) == [0, 2, 3, 5, 6, 7, 4]
    assert n == 6 and list(ids) == [10, -1, 11, 12, 13, 14, 15]
    assert out["valid_mask"].sum() == 7 and not out["valid_mask"][2]  # proposal 1 (slot 2) was masked
    assert out["primitive_ids"][4] == 15 and out["weights"][4] == 2.0


def test_oracle_cull_threshold_and_max_primitives():
    t = O.empty_tile(6, L)
    t["valid_mask"][:5] = True
    t["weights"][:] = [0.5, 1e-5, 0.3, 0.9, 0.2, 7.0]
    out, n, mass = O.primitive_map_cull(t, 1e-4)
    assert n == 1 and mass == 1e-5 and not out["valid_mask"][1]
    # threshold = the (max_primitives+1)-th largest weight (0.3), culled strictly below it: the
    # reference keeps max_primitives + 1 here (primitive_map.py:1222-1229)
    out, n, mass = O.primitive_map_cull(t, 1e-4, max_primitives=2)
    assert n == 2 and np.isclose(mass, 1e-5 + 0.2)
    assert list(np.flatnonzero(out["valid_mask"])) == [0, 2, 3]


def test_oracle_recency_and_forget():
    t = O.empty_tile(4, L)
    t["valid_mask"][:3] = True
    t["last_supported_scan_seq"][:] = [10, 0, 12, 0]
    t["Lambdas"][:] = np.eye(3)
    t["thetas"][:] = 1.0
    t["weights"][:] = 2.0
    out, (nv, down, tr) = O.primitive_map_recency_inflate(t, 10, 0.02, 0.05)
    d = np.array([1.0, np.exp(-0.2), 1.0, 1.0])
    np.testing.assert_allclose(out["Lambdas"][:, 0, 0], d)
    assert nv == 3.0 and np.isclose(down, 1 - d[1]) and np.isclose(tr, 1 / d[1] - 1)
    out, (_, _, _) = O.primitive_map_recency_inflate(t, 1000, 0.02, 0.05)
    assert np.isclose(out["thetas"][1, 0], 0.05)  # clipped at min_scale
    assert np.all(O.primitive_map_forget(t, 0.995)["weights"] == 0.995 * 2.0)


# ----------------------------------------------------------------------------------- GPU
def _random_tile(rng, M, frac_valid=0.7):
    t = O.empty_tile(M, L)
    B = rng.normal(size=(M, 3, 3))
    t["Lambdas"] = B @ np.swapaxes(B, 1, 2) + 0.5 * np.eye(3)
    t["thetas"] = rng.normal(size=(M, 3)) * 3.0
    t["etas"] = rng.normal(size=(M, L, 3))
    t["weights"] = rng.uniform(0, 1, M) ** 3
    t["timestamps"] = rng.uniform(0, 5, M)
    t["created_timestamps"] = rng.uniform(0, 5, M)
    t["last_supported_scan_seq"] = rng.integers(0, 40, M).astype(np.int64)
    t["last_update_scan_seq"] = rng.integers(0, 40, M).astype(np.int64)
    t["primitive_ids"] = rng.permutation(M).astype(np.int64)
    t["valid_mask"] = rng.uniform(0, 1, M) < frac_valid
    t["cam_mass"] = rng.uniform(0, 1, M) * (rng.uniform(0, 1, M) > 0.5)
    t["lidar_mass"] = rng.uniform(0, 1, M)
    t["rgb_cam_accum"] = rng.uniform(0, 1, (M, 3))
    t["rgb_cam_denom"] = rng.uniform(0, 1, M)
    return t


def _upload(dm, tile_id, tile):
    s0, n = dm.tile_range(tile_id)
    cur = dm.download()
    for k, v in tile.items():
        a = cur[k]
        a[s0:s0 + n] = v.astype(a.dtype) if k == "valid_mask" else v
        dm.upload(**{k: a})


def _compare(dm, tile_id, ref, rtol=1e-12):
    got = dm.download_tile(tile_id)
    for k, v in ref.items():
        g = got[k]
        if k in ("valid_mask", "primitive_ids", "last_supported_scan_seq", "last_update_scan_seq"):
            np.testing.assert_array_equal(g.astype(v.dtype), v, err_msg=k)
        else:
            np.testing.assert_allclose(g, v, rtol=rtol, atol=rtol * max(1.0, float(np.max(np.abs(v)))), err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("packed", [True, False])
def test_gpu_map_maintenance_sequence_matches_oracle(ctx, packed):
    """recency -> cull(max_primitives) -> insert_masked -> merge_reduce -> forget on tile 1 of a
    3-tile map; tiles 0 and 2 must stay untouched (either device layout)."""
    from gcslam import primitive_map as PM
    rng = np.random.default_rng(42)
    M = 300
    dm = PM.DevicePrimitiveMap(3, M, ctx=ctx, packed=packed)
    tiles = [_random_tile(rng, M) for _ in range(3)]
    for t_id, t in enumerate(tiles):
        _upload(dm, t_id, t)
    ref = tiles[1]
    _, _, eff, st = PM.primitive_map_recency_inflate(dm, [1], 37, 0.02, 0.05)
    ref, rst = O.primitive_map_recency_inflate(ref, 37, 0.02, 0.05)
    _compare(dm, 1, ref)
    assert eff.realized == rst[0]
    np.testing.assert_allclose(st.stale_precision_downscale_total, rst[1], rtol=1e-12)
    np.testing.assert_allclose(st.staleness_cov_inflation_trace, rst[2], rtol=1e-12)
    res, cert, _ = PM.primitive_map_cull(dm, 1, 1e-3, max_primitives=150)
    ref, n_c, mass = O.primitive_map_cull(ref, 1e-3, max_primitives=150)
    assert res.n_culled == n_c and not cert.exact
    np.testing.assert_allclose(res.mass_dropped, mass, rtol=1e-12)
    _compare(dm, 1, ref)
    K = 64
    mask = rng.uniform(0, 1, K) < 0.8
    B = rng.normal(size=(K, 3, 3))
    props = dict(Lambdas=B @ np.swapaxes(B, 1, 2) + np.eye(3), thetas=rng.normal(size=(K, 3)),
                 etas=rng.normal(size=(K, L, 3)), weights=rng.uniform(0.1, 1, K), colors=rng.uniform(-0.1, 1.1, (K, 3)),
                 sources=rng.integers(0, 2, K))
    dm.next_global_id = 1000
    res, _, _ = PM.primitive_map_insert_masked(dm, 1, props["Lambdas"], props["thetas"], props["etas"],
                                               props["weights"], 4.5, mask, scan_seq=38, colors_new=props["colors"],
                                               sources_new=props["sources"])
    ref, n_i, ids, slots = O.primitive_map_insert_masked(ref, props["Lambdas"], props["thetas"], props["etas"],
                                                         props["weights"], 4.5, mask, 38, 0.02, 1000, props["colors"],
                                                         props["sources"])
    assert res.n_inserted == n_i and dm.next_global_id == 1000 + n_i
    np.testing.assert_array_equal(res.target_slots, slots)
    np.testing.assert_array_equal(res.new_ids, ids)
    _compare(dm, 1, ref)
    res, _, _ = PM.primitive_map_merge_reduce(dm, 1, merge_threshold=2.0, max_pairs=16)
    ref, n_m = O.primitive_map_merge_reduce(ref, 2.0, 16)
    assert res.n_merged == n_m and n_m > 0
    _compare(dm, 1, ref, rtol=1e-10)
    PM.primitive_map_forget(dm, 1, 0.995)
    ref = O.primitive_map_forget(ref, 0.995)
    _compare(dm, 1, ref, rtol=1e-10)
    for t_id in (0, 2):
        _compare(dm, t_id, tiles[t_id], rtol=0.0)


@pytest.mark.gpu
def test_gpu_merge_reduce_close_pair_kat(ctx):
    """test_primitive_map_merge_reduce.py:76-99 on the device."""
    from gcslam import primitive_map as PM
    dm = PM.DevicePrimitiveMap(1, 3, ctx=ctx)
    _upload(dm, 0, _merge_kat_tile())
    dm.total_count = 3
    res, cert, eff = PM.primitive_map_merge_reduce(dm, 0, merge_threshold=0.5, max_pairs=1, max_tile_size=10)
    got = dm.download("weights", "valid_mask")
    assert res.n_merged == 1 and cert.frobenius_applied and eff.realized == 1.0
    assert list(got["valid_mask"]) == [1, 0, 1] and np.isclose(got["weights"][0], 2.0)
    assert dm.total_count == 2


@pytest.mark.gpu
@pytest.mark.parametrize("first,second,expect", [
    (([1.0, 0.0, 0.0], 0), ([0.2, 0.2, 0.2], 1), [1.0, 0.0, 0.0]),
    (([0.2, 0.2, 0.2], 1), ([0.0, 1.0, 0.0], 0), [0.0, 1.0, 0.0]),
])
def test_gpu_color_provenance_kat(ctx, first, second, expect):
    """test_map_color_provenance.py:72-87: device insert_masked then device fuse."""
    from gcslam import primitive_map as PM
    dm = PM.DevicePrimitiveMap(1, 1, ctx=ctx)
    res, _, _ = PM.primitive_map_insert_masked(dm, 0, np.eye(3)[None], np.zeros((1, 3)), np.zeros((1, L, 3)),
                                               np.array([1.0]), 0.0, np.array([True]), scan_seq=0,
                                               colors_new=np.array([first[0]]), sources_new=np.array([first[1]]))
    assert res.n_inserted == 1 and res.new_ids[0] == 0
    PM.primitive_map_fuse(dm, 0, np.array([0]), np.eye(3)[None], np.zeros((1, 3)), np.zeros((1, L, 3)),
                          np.array([1.0]), np.array([1.0]), 1.0, 1, valid_mask=np.array([True]),
                          colors_meas=np.array([second[0]]), sources_meas=np.array([second[1]]))
    np.testing.assert_allclose(dm.download("rgb")["rgb"][0], expect, atol=1e-6)


@pytest.mark.gpu
def test_gpu_map_ops_edge_cases(ctx):
    from gcslam import primitive_map as PM
    dm = PM.DevicePrimitiveMap(2, 16, ctx=ctx)
    res, cert, _ = PM.primitive_map_cull(dm, 0)                   # empty tile: exact no-op
    assert res.n_culled == 0 and cert.exact
    res, cert, _ = PM.primitive_map_merge_reduce(dm, 1)           # < 2 valid: no-op
    assert res.n_merged == 0 and cert.exact
    _, _, _, st = PM.primitive_map_recency_inflate(dm, [0, 1], 5)
    assert st.staleness_inflation_strength == 0.0
    with pytest.raises(ValueError):
        PM.primitive_map_insert_masked(dm, 0, np.zeros((17, 3, 3)), np.zeros((17, 3)), np.zeros((17, L, 3)),
                                       np.ones(17), 0.0, np.ones(17, bool))       # K > m_tile
    with pytest.raises(ValueError):
        PM.primitive_map_forget(dm, 5)
    big = PM.DevicePrimitiveMap(1, 40, ctx=ctx)
    _upload(big, 0, _random_tile(np.random.default_rng(1), 40, 1.0))
    res, cert, _ = PM.primitive_map_merge_reduce(big, 0, max_tile_size=20)  # budget cap
    assert res.n_merged == 0 and "merge_reduce_budget_cap" in cert.approximation_triggers
