"""Map view extraction + OT association: extract_atlas_map_view
(structures/primitive_map.py:356-451) and associate_primitives_ot
(operators/primitive_association.py:239-553).

The reference's one test for this path is the budget-assertion test
(test/test_budget_assertions.py:91-140), restated below for the device. Everything else is pinned
by the oracle restatement ("parity unpinned" against reference outputs): candidate indices, tile
ids and slots must match the oracle exactly; costs within 1e-10 relative; the Sinkhorn outputs
(50 fixed iterations of powers 1/6) within 1e-8 relative."""

import numpy as np
import pytest

from oracle import gc_oracle as O

L = 3


def test_oracle_tiling_helpers():
    assert O.hex_disk_axial(1) == [(-1, 0), (-1, 1), (0, -1), (0, 0), (0, 1), (1, -1), (1, 0)]
    assert len(O.hex_disk_axial(2)) == 19
    # bias 2^20 then a 21-bit mask per axis (tiling.py:91-105)
    assert int(O.tile_ids_from_cells(0, 0, 0)) == ((1 << 20) << 42) | ((1 << 20) << 21) | (1 << 20)
    assert int(O.tile_ids_from_cells(-1, 2, -3)) == (((1 << 20) - 1) << 42) | (((1 << 20) + 2) << 21) | ((1 << 20) - 3)


def test_oracle_view_topk_order():
    t = O.empty_tile(6, L)
    t["valid_mask"][[0, 2, 3, 5]] = True
    t["weights"][:] = [0.2, 9.0, 0.7, 0.2, 5.0, 0.9]  # slots 1, 4 invalid despite their weight
    v = O.extract_atlas_map_view({7: t}, [7, 8], 4, 6)
    assert list(v["candidate_slots"][:4]) == [5, 2, 0, 3]      # by weight, tie 0.2 by slot
    assert list(v["candidate_slots"][4:]) == [0, 1, 2, 3]      # missing tile 8: empty, slot order
    assert list(v["candidate_tile_ids"]) == [7] * 4 + [8] * 4 and not v["valid_mask"][4:].any()


def _hex_map(rng, m_tile, n_valid, cells):
    tiles = {}
    for (c1, c2, cz) in cells:
        t = O.empty_tile(m_tile, L)
        n = n_valid
        # points inside the cell's parallelogram: s1 = x in [c1 h, c1 h + h), s2 = x/2 + y √3/2
        s1 = rng.uniform(c1 * 2.0, c1 * 2.0 + 2.0, n)
        s2 = rng.uniform(c2 * 2.0, c2 * 2.0 + 2.0, n)
        x, y = s1, (s2 - 0.5 * s1) / (np.sqrt(3.0) * 0.5)
        z = rng.uniform(cz * 2.0, cz * 2.0 + 2.0, n)
        pos = np.column_stack([x, y, z])
        B = rng.normal(size=(n, 3, 3)) * 0.3
        Lam = B @ np.swapaxes(B, 1, 2) + 2.0 * np.eye(3)
        t["Lambdas"][:n] = Lam
        t["thetas"][:n] = np.einsum("nij,nj->ni", Lam, pos)
        t["etas"][:n] = rng.normal(size=(n, L, 3)) * 2.0
        t["weights"][:n] = rng.uniform(0.1, 1.0, n)
        t["valid_mask"][:n] = rng.uniform(0, 1, n) < 0.9
        t["primitive_ids"][:n] = rng.permutation(n)
        t["last_supported_scan_seq"][:n] = rng.integers(0, 12, n)
        tiles[int(O.tile_ids_from_cells(c1, c2, cz))] = t
    return tiles


def _meas(rng, N, lo=-2.0, hi=4.0):
    pos = rng.uniform(lo, hi, (N, 3))
    pos[:, 2] = rng.uniform(0.0, 2.0, N)
    Lam = np.tile(4.0 * np.eye(3), (N, 1, 1))
    return dict(Lambdas=Lam, thetas=4.0 * pos, etas=rng.normal(size=(N, L, 3)) * 2.0,
                weights=rng.uniform(0.1, 1.0, N), valid_mask=rng.uniform(0, 1, N) < 0.85)


def test_oracle_association_self_match():
    rng = np.random.default_rng(3)
    tiles = _hex_map(rng, 16, 16, [(0, 0, 0)])
    tid = list(tiles)[0]
    tiles[tid]["valid_mask"][:] = True
    view = O.extract_atlas_map_view(tiles, [tid], 16, 16)
    j = 5  # a measurement identical to view entry j: its best candidate, cost 0 after the row min
    meas = dict(Lambdas=np.linalg.inv(view["covariances"][j:j + 1]) - O.EPS_LIFT * np.eye(3),
                thetas=None, etas=view["etas"][j:j + 1], weights=np.ones(1), valid_mask=np.ones(1, bool))
    meas["thetas"] = np.einsum("nij,nj->ni", meas["Lambdas"] + O.EPS_LIFT * np.eye(3), view["positions"][j:j + 1])
    res, cert = O.associate_primitives_ot(meas, view, dict(scan_seq=0, recency_decay_lambda=0.0))
    assert res["candidate_pool_indices"][0, 0] == j and abs(res["cost_matrix"][0, 0]) < 1e-12
    assert cert["nonzero_a"] == 1 and res["row_masses"][0] > 0


# ----------------------------------------------------------------------------------- GPU
def _device_map(ctx, tiles, m_tile, extra_dense=1):
    from gcslam.primitive_map import DevicePrimitiveMap
    keys = list(tiles) + [-(i + 1) for i in range(extra_dense)]  # plus unlisted dense tiles
    dm = DevicePrimitiveMap(len(keys), m_tile, ctx=ctx)
    dm.set_tile_keys(keys)
    full = {k: np.concatenate([tiles[kk][k] if kk in tiles else O.empty_tile(m_tile, L)[k] for kk in keys])
            for k in O.empty_tile(1, L)}
    full["valid_mask"] = full["valid_mask"].astype(np.uint8)
    dm.upload(**full)
    return dm


def _cmp(got, ref, exact, rtol):
    for k, v in ref.items():
        if k not in got:
            continue
        g = np.asarray(got[k])
        if k in exact:
            np.testing.assert_array_equal(g.astype(np.asarray(v).dtype), v, err_msg=k)
        else:
            v = np.asarray(v, np.float64)
            np.testing.assert_allclose(g, v, rtol=rtol, atol=rtol * max(1.0, float(np.max(np.abs(v)))), err_msg=k)


@pytest.mark.gpu
def test_gpu_map_view_matches_oracle(ctx):
    from gcslam.association import extract_atlas_map_view
    rng = np.random.default_rng(11)
    cells = [(a, b, 0) for a in range(-1, 3) for b in range(-1, 3)]
    tiles = _hex_map(rng, 96, 80, cells)
    dm = _device_map(ctx, tiles, 96)
    ids = list(tiles)[:9] + [int(O.tile_ids_from_cells(40, 40, 0))]  # the last one is missing
    view = extract_atlas_map_view(dm, ids, 48)
    ref = O.extract_atlas_map_view(tiles, ids, 48, 96)
    got = view.download()
    _cmp(got, {k: v for k, v in ref.items() if k not in ("tile_ids", "m_tile_view")},
         ("candidate_tile_ids", "candidate_slots", "valid_mask", "primitive_ids", "last_supported_scan_seq"), 1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("wprop", [False, True])
def test_gpu_association_matches_oracle(ctx, wprop):
    from gcslam.association import (AssociationConfig, MeasurementMassPolicy, associate_primitives_ot,
                                    extract_atlas_map_view)
    rng = np.random.default_rng(5 + wprop)
    cells = [(a, b, 0) for a in range(-2, 3) for b in range(-2, 3)]
    tiles = _hex_map(rng, 64, 60, cells)
    dm = _device_map(ctx, tiles, 64)
    ids = list(tiles)
    view = extract_atlas_map_view(dm, ids, 32)
    ref_view = O.extract_atlas_map_view(tiles, ids, 32, 64)
    meas = _meas(rng, 300)
    cfg = AssociationConfig(scan_seq=9, a_policy=MeasurementMassPolicy.WEIGHT_PROPORTIONAL if wprop else
                            MeasurementMassPolicy.UNIFORM)

    class Batch:
        pass

    b = Batch()
    for k, v in meas.items():
        setattr(b, k, v)
    res, cert, eff = associate_primitives_ot(b, view, cfg)
    ref, rc = O.associate_primitives_ot(meas, ref_view, dict(scan_seq=9, weight_proportional=wprop))
    got = dict(res.__dict__)
    _cmp(got, {k: ref[k] for k in ("candidate_pool_indices", "candidate_tile_ids", "candidate_slots")},
         ("candidate_pool_indices", "candidate_tile_ids", "candidate_slots"), 0.0)
    _cmp(got, {"cost_matrix": ref["cost_matrix"]}, (), 1e-10)
    _cmp(got, {k: ref[k] for k in ("responsibilities", "row_masses")}, (), 1e-8)
    ot = cert.ot
    for k in ("marginal_defect_a", "marginal_defect_b", "transport_mass_total", "sum_a", "sum_m", "sum_novel"):
        np.testing.assert_allclose(getattr(ot, k), rc[k], rtol=1e-8, atol=1e-12, err_msg=k)
    np.testing.assert_allclose(cert.support.ess_total, rc["ess"], rtol=1e-8)
    np.testing.assert_allclose(eff.realized, rc["total_cost"], rtol=1e-8)
    assert ot.nonzero_a == rc["nonzero_a"] and ot.nonzero_b == rc["nonzero_b"]
    assert "sinkhorn_fixed_iter" in cert.approximation_triggers


@pytest.mark.gpu
def test_gpu_association_budget_kat(ctx):
    """test_budget_assertions.py:91-140: K_ASSOC measurements and map primitives at the origin,
    one tile keyed 0, the reference's compute-cert budgets."""
    from gcslam.association import AssociationConfig, associate_primitives_ot, extract_atlas_map_view
    from gcslam.primitive_map import DevicePrimitiveMap
    K = 8
    dm = DevicePrimitiveMap(1, K, ctx=ctx)
    eta = np.zeros((K, L, 3))
    eta[:, 0] = [1.0, 0.0, 0.0]
    dm.upload(Lambdas=np.tile(np.eye(3), (K, 1, 1)), etas=eta, weights=np.ones(K),
              primitive_ids=np.arange(K, dtype=np.int64), valid_mask=np.ones(K, np.uint8))
    view = extract_atlas_map_view(dm, [0], K)

    class Batch:
        Lambdas = np.tile(np.eye(3), (K, 1, 1))
        thetas = np.zeros((K, 3))
        etas = eta
        weights = np.ones(K)
        valid_mask = np.ones(K, bool)

    _, cert, _ = associate_primitives_ot(Batch, view, AssociationConfig(k_assoc=K, k_sinkhorn=50))
    assert cert.compute.largest_tensor_shape[0] <= K and cert.compute.largest_tensor_shape[1] <= K
    assert cert.compute.segment_sum_k == K
    assert cert.compute.alloc_bytes_est <= K * K * 8 * 4
    assert cert.compute.psd_projection_count <= view.count


@pytest.mark.gpu
def test_gpu_association_empty_inputs(ctx):
    from gcslam.association import associate_primitives_ot, extract_atlas_map_view
    rng = np.random.default_rng(2)
    tiles = _hex_map(rng, 16, 16, [(0, 0, 0)])
    dm = _device_map(ctx, tiles, 16)
    view = extract_atlas_map_view(dm, list(tiles), 8)
    meas = _meas(rng, 10)
    meas["valid_mask"][:] = False

    class Batch:
        pass

    for k, v in meas.items():
        setattr(Batch, k, v)
    res, cert, eff = associate_primitives_ot(Batch, view)
    assert cert.exact and eff.realized == 0.0 and not res.responsibilities.any() and not res.row_masses.any()
