"""The C5 in-scan PrimitiveMap update (csrc/gc_scanmap.hip; build-defined, parity unpinned — the
reference's step 12b, pipeline.py:1236-1327, fuses a measurement batch built outside this path).

Every budgeted point, deskewed with hypothesis 0's twist, is one world-frame Gaussian row (pose
z_t of hypothesis 0, t_z = 0, Σ_lidar inflated by J Σ_pose Jᵀ) fused into the slot hashed from its
voxel. The oracle rebuilds the rows from the raw scan and the pose block the GPU used
(gc_pipeline_get_scan_map_pose), fuses them with its np.add.at restatement of primitive_map_fuse
and must agree: slot keys, touched-slot count, timestamps, scan sequences, camera mass and colours
exactly; Λ, θ, η, w and LiDAR mass within 1e-12 of each field's largest entry (the rows' 3x3
inverse and products round differently in NumPy, and the device sums each slot's rows in a fixed
tree order where np.add.at adds them one by one). The pose block itself is the pipeline's own
hypothesis-0 result (ξ and Σ_post bit-identical to the per-hypothesis getters), which the config
tests compare with the oracle at the north-star bars.
"""

import numpy as np
import pytest

from oracle import cases
from oracle import gc_oracle as O
from test_gpu_configs import _pipeline

pytestmark = pytest.mark.gpu

FIELDS_CLOSE = ("Lambdas", "thetas", "etas", "weights", "lidar_mass")
FIELDS_EXACT = ("timestamps", "last_supported_scan_seq", "last_update_scan_seq", "cam_mass", "rgb", "colors",
                "rgb_cam_accum", "rgb_cam_denom")


def _map(ctx, M, seed):
    from gcslam.primitive_map import DevicePrimitiveMap
    rng = np.random.default_rng(seed)
    B = rng.normal(size=(M, 3, 3))
    dm = DevicePrimitiveMap(1, M, ctx=ctx)
    dm.upload(Lambdas=B @ np.swapaxes(B, 1, 2) + np.eye(3), thetas=rng.normal(size=(M, 3)),
              etas=rng.normal(size=(M, 3, 3)), weights=rng.uniform(0, 2, M), timestamps=rng.uniform(0, 5, M),
              lidar_mass=rng.uniform(0, 1, M))
    return dm


def _check_scan(pipe, dm, tile0, s, k, cap, M, voxel, iw):
    """iw: the pipeline's IW state before the scan (Σ_lidar of the update is the LiDAR mode the scan
    started from, before its own measurement-IW apply)."""
    zt, Sp, xi = pipe.scan_map_pose()
    _, _, xi_all = pipe.bin_stats()
    _, _, Sig = pipe.hyp_stats()
    assert np.array_equal(xi, xi_all[0]), "pose block: ξ is not hypothesis 0's"
    assert np.array_equal(Sp, Sig[0][0:6, 0:6]), "pose block: Σ_pose is not hypothesis 0's Σ_post"
    h0 = np.concatenate([zt, Sp.reshape(-1), xi])
    rows = O.scan_map_rows(s["points"], s["timestamps"], s["weights"], cap, s["scan_start"], s["scan_end"], h0,
                           iw["nu_meas"], iw["Psi_meas"], np.asarray(pipe.cfg.lidar_origin), voxel, M)
    ref, nref = O.scan_map_update(tile0, rows, s["scan_end"], k)
    got = dm.download()
    assert pipe.scan_map_count() == nref, f"scan{k}: touched slots {pipe.scan_map_count()} vs {nref}"
    for f in FIELDS_EXACT:
        assert np.array_equal(got[f], ref[f]), f"scan{k} {f}"
    for f in FIELDS_CLOSE:
        scale = np.max(np.abs(ref[f]))
        err = np.max(np.abs(got[f] - ref[f]))
        assert err <= 1e-12 * scale, f"scan{k} {f}: {err:.3e} vs scale {scale:.3e}"
    return nref


@pytest.mark.parametrize("n_az,cap,M", [(1024, 16384, 1 << 14), (8192, 65536, 1 << 20)])
def test_scan_map_update_matches_oracle(ctx, n_az, cap, M):
    """Small map, and the C5 geometry: 131,072-point scans budgeted to 65,536 rows into 1,048,576 slots."""
    voxel = 0.1
    case = cases.build(H=8, n_az=n_az, n_scans=2, io="computed", cap=cap)
    pipe = _pipeline(case, ctx, 8, cap, True)
    dm = _map(ctx, M, n_az)
    pipe.attach_primitive_map(dm, voxel)
    touched = []
    for k, s in enumerate(case["scans"]):
        tile0, iw0 = dm.download(), pipe.get_iw()
        pipe.stage_scan(0, s)
        pipe.run_scan(0, s, k)
        touched.append(_check_scan(pipe, dm, tile0, s, k, cap, M, voxel, iw0))
    assert all(t > 1000 for t in touched), touched
    pipe.close()


def test_scan_map_colours_recomputed_after_host_writes(ctx):
    """The map's colours stop being the fuse's estimate when a host operation writes colour fields
    (a colour upload before scan 1, a camera-sourced insert before scan 2): the next in-scan update
    recomputes rgb / colors on every slot, as primitive_map_fuse does on every fuse
    (primitive_map.py:1097-1105), and the map reports its colours current afterwards."""
    from gcslam.primitive_map import primitive_map_insert_masked
    voxel, cap, M = 0.1, 16384, 1 << 14
    case = cases.build(H=4, n_az=1024, n_scans=3, io="computed", cap=cap)
    pipe = _pipeline(case, ctx, 4, cap, True)
    dm = _map(ctx, M, 11)
    rng = np.random.default_rng(12)
    den = rng.uniform(0.0, 2.0, M) * (rng.uniform(size=M) > 0.3)
    dm.upload(cam_mass=den, rgb_cam_denom=den, rgb_cam_accum=rng.uniform(0, 1.5, (M, 3)) * den[:, None])
    pipe.attach_primitive_map(dm, voxel)
    for k, s in enumerate(case["scans"]):
        if k == 1:
            dm.upload(rgb=rng.uniform(size=(M, 3)), colors=rng.uniform(size=(M, 3)))
            assert not dm.colors_current
        if k == 2:
            K = 64
            Bq = rng.normal(size=(K, 3, 3))
            primitive_map_insert_masked(dm, 0, Bq @ np.swapaxes(Bq, 1, 2) + np.eye(3), rng.normal(size=(K, 3)),
                                        rng.normal(size=(K, 3, 3)), rng.uniform(0.5, 2.0, K), 7.0, np.ones(K, bool),
                                        scan_seq=k, colors_new=rng.uniform(0.2, 3.0, (K, 3)),
                                        sources_new=np.zeros(K, np.int32))
            assert not dm.colors_current
        tile0, iw0 = dm.download(), pipe.get_iw()
        pipe.stage_scan(0, s)
        pipe.run_scan(0, s, k)
        _check_scan(pipe, dm, tile0, s, k, cap, M, voxel, iw0)
        assert dm.colors_current
    pipe.close()


def test_scan_map_update_replicated_across_shards(ctx):
    """Two shards (4 + 4 of 8, chunk geometry as for 8) each with its own copy of the map and
    host-gathered records: both maps end bit-identical to the unsharded pipeline's."""
    case = cases.build(H=8, n_az=1024, n_scans=2, io="computed")
    cap = case["n"]
    full = _pipeline(case, ctx, 8, cap, True)
    shards = [_pipeline(case, ctx, 8, cap, True, rank=r, world=2, geometry_hyps=8) for r in range(2)]
    maps = [_map(ctx, 1 << 14, 3) for _ in range(3)]
    full.attach_primitive_map(maps[0], 0.1)
    for p, m in zip(shards, maps[1:]):
        p.attach_primitive_map(m, 0.1)
        p.set_scan_map_mode(replicated=True)
    for k, s in enumerate(case["scans"]):
        full.stage_scan(0, s)
        full.run_scan(0, s, k)
        for p in shards:
            p.stage_scan(0, s)
            p.run_scan_local(0, s, k)
        recs = np.stack([p.partial() for p in shards])
        for p in shards:
            p.finish_scan(recs)
        ctx.sync()
        ref = maps[0].download()
        for m in maps[1:]:
            got = m.download()
            for f in ref:
                assert np.array_equal(got[f], ref[f]), f"scan{k} {f}"


def test_scan_map_update_runs_on_the_owner_rank_only(ctx):
    """The default scan-map mode (GC_SMAP_OWNER): of two shards (4 + 4 of 8), only hypothesis 0's
    rank runs the update (backend_node.py:2081-2083); its map ends bit-identical to the unsharded
    pipeline's, the other rank's map is left exactly as uploaded and reports no touched slots, and the
    other rank's slot rotation (no map update as the slot's last reader) stays usable."""
    case = cases.build(H=8, n_az=1024, n_scans=3, io="computed")
    cap = case["n"]
    full = _pipeline(case, ctx, 8, cap, True)
    shards = [_pipeline(case, ctx, 8, cap, True, rank=r, world=2, geometry_hyps=8) for r in range(2)]
    maps = [_map(ctx, 1 << 14, 3) for _ in range(3)]
    untouched = maps[2].download()
    full.attach_primitive_map(maps[0], 0.1)
    for p, m in zip(shards, maps[1:]):
        p.attach_primitive_map(m, 0.1)
    assert shards[0].scan_map_owner() and not shards[1].scan_map_owner()
    for k, s in enumerate(case["scans"]):
        full.stage_scan(k % 2, s)
        full.run_scan(k % 2, s, k)
        for p in shards:
            p.stage_scan(k % 2, s)
            p.run_scan_local(k % 2, s, k)
        recs = np.stack([p.partial() for p in shards])
        for p in shards:
            p.finish_scan(recs)
        ref, own, other = maps[0].download(), maps[1].download(), maps[2].download()
        for f in ref:
            assert np.array_equal(own[f], ref[f]), f"scan{k} owner {f}"
            assert np.array_equal(other[f], untouched[f]), f"scan{k} non-owner {f} changed"
        assert shards[0].scan_map_count() == full.scan_map_count() > 0
        assert shards[1].scan_map_count() == 0
    for p in [full] + shards:
        p.close()


def test_first_pipelines_map_read_after_a_later_pipelines_finish(ctx):
    """Several pipelines with attached maps on one context: each scan_finish chains its
    side-stream update after the context's pending one, so reading the FIRST pipeline's map after a
    later pipeline's finish (no ctx.sync in between) joins every update, and the map matches the
    oracle."""
    voxel, cap, M = 0.1, 16384, 1 << 14
    case = cases.build(H=4, n_az=1024, n_scans=2, io="computed", cap=cap)
    pipes = [_pipeline(case, ctx, 4, cap, True) for _ in range(3)]
    maps = [_map(ctx, M, 21 + i) for i in range(3)]
    for p, m in zip(pipes, maps):
        p.attach_primitive_map(m, voxel)
    for k, s in enumerate(case["scans"]):
        tiles, iws = [m.download() for m in maps], [p.get_iw() for p in pipes]
        for p in pipes:
            p.stage_scan(0, s)
            p.run_scan(0, s, k)
        for i in (0, 1):  # the earlier pipelines' maps, read right after the last pipeline's finish
            _check_scan(pipes[i], maps[i], tiles[i], s, k, cap, M, voxel, iws[i])
    for p in pipes:
        p.close()


def test_scan_map_attach_rules(ctx):
    from gcslam.primitive_map import DevicePrimitiveMap
    case = cases.build(H=2, n_az=256, n_scans=1, io="computed")
    pipe = _pipeline(case, ctx, 2, case["n"], True)
    dm = DevicePrimitiveMap(1, 1024, ctx=ctx)
    with pytest.raises(ValueError, match="voxel"):
        pipe.attach_primitive_map(dm, 0.0)
    with pytest.raises(ValueError, match="no PrimitiveMap"):
        pipe.scan_map_count()
    s = case["scans"][0]
    pipe.attach_primitive_map(dm, 0.2)
    pipe.stage_scan(0, s)
    pipe.run_scan_local(0, s, 0)
    with pytest.raises(ValueError, match="pending"):
        pipe.attach_primitive_map(None)
    with pytest.raises(ValueError, match="map update"):  # its slot is still to be read by scan_finish
        pipe.stage_scan(0, s)
    pipe.stage_scan(1, s)
    pipe.finish_scan()
    assert pipe.scan_map_count() > 0
    pipe.attach_primitive_map(None)
    w0 = dm.download("weights")["weights"]
    pipe.stage_scan(0, s)
    pipe.run_scan(0, s, 1)
    ctx.sync()
    assert np.array_equal(dm.download("weights")["weights"], w0)  # detached: no update
