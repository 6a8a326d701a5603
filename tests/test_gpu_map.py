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


@pytest.mark.parametrize("K,M,world", [(5000, 1 << 12, False), (20000, 1 << 16, False), (3000, 2000, True),
                                       (1, 10, False), (131072, 1 << 20, False), (131072, 1 << 20, True)])
def test_primitive_map_fuse_matches_oracle(ctx, K, M, world):
    from gcslam.primitive_map import DevicePrimitiveMap, fuse_rows
    rng = np.random.default_rng(K + M)
    c, tile = _case(rng, K, M), _tile(rng, M)
    dm = DevicePrimitiveMap(1, M, ctx=ctx)
    dm.upload(**tile)
    pose = np.array([1.0, -2.0, 0.0, 0.05, -0.02, 0.7]) if world else None
    n = fuse_rows(dm, c["slots"], c["Lambdas"], c["thetas"], c["etas"], c["weights"], c["resp"], 7.5, 11,
                  c["valid"], c["colors"], c["sources"], world_pose=pose)
    Lm, th, et = c["Lambdas"], c["thetas"], c["etas"]
    if world:
        Lm, th, et = O.transform_gaussian_to_world(Lm, th, et, pose)
    ref, nref = O.primitive_map_fuse(tile, c["slots"], Lm, th, et, c["weights"], c["resp"], 7.5, 11, c["valid"],
                                     c["colors"], c["sources"])
    got = dm.download()
    assert n == nref
    for k, v in ref.items():
        if world and k in ("Lambdas", "thetas", "etas"):
            np.testing.assert_allclose(got[k], v, rtol=1e-12, atol=1e-12 * np.max(np.abs(v)), err_msg=k)
        else:
            np.testing.assert_array_equal(got[k], v, err_msg=k)


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
