"""The per-scan hypothesis exchange on the device (backend_node.py:2036-2119).

A rank's scan is gc_pipeline_scan_local (a1-a15 + its partial record) followed by
gc_pipeline_scan_finish (exchange, fixed rank-order reduction in k_combine_final, barycenter, IW
apply, Q, map update). These tests run the G > 1 reduction of k_combine_final on the GPU:

  * two hypothesis shards (H = 8 as 4 + 4) in one process, records gathered on the host;
  * the same over two processes on one GPU with a gloo all-gather of the device records;
  * the RCCL path with a single-rank communicator (ncclAllGather inside the pipeline).

Bars: the combined belief, IW state, Q and map are bit-identical across ranks, and within 1e-12
relative of the unsharded pipeline (the shard sums associate like the unsharded tree).
"""

import os
import sys

import numpy as np
import pytest

from oracle import cases

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _state(pipe):
    c, iw, mp, b = pipe.combined(), pipe.get_iw(), pipe.get_map(), pipe.get_beliefs()
    return dict(comb_L=c["L"], comb_h=c["h"], comb_z=c["z_lin"], comb_X=c["X_anchor"], nu_proc=iw["nu_proc"],
                Psi_proc=iw["Psi_proc"], nu_meas=iw["nu_meas"], Psi_meas=iw["Psi_meas"], Q=iw["Q"], map=mp["map"],
                map_der=mp["derived"], L=b["L"], h=b["h"], X=b["X_anchor"])


SHARED = ("comb_L", "comb_h", "comb_z", "comb_X", "nu_proc", "Psi_proc", "nu_meas", "Psi_meas", "Q", "map", "map_der")


def _make(case, ctx, rank, world):
    from gcslam.pipeline import BatchedScanPipeline, PipelineConfig
    H = case["hyp"]["weights"].shape[0]
    pipe = BatchedScanPipeline(H, case["n"], PipelineConfig(n_points_cap=case["n"]), rank=rank, world_size=world,
                               ctx=ctx)
    sl = slice(pipe.h0, pipe.h1)
    hy = case["hyp"]
    pipe.set_beliefs(hy["X_anchor"][sl], hy["z_lin"][sl], hy["L"][sl], hy["h"][sl], hy["stamp"][sl])
    pipe.set_weights(hy["weights"])
    Lio, hio, cert = case["io"]
    pipe.set_io_evidence(Lio[sl], hio[sl], cert[sl])
    pipe.set_iw(*case["iw"])
    pipe.set_map(case["map_record"])
    return pipe


def _rel_close(a, b, rel, what):
    err = np.max(np.abs(a - b))
    scale = max(np.max(np.abs(b)), 1e-300)
    assert err <= rel * scale, f"{what}: {err:.3e} vs scale {scale:.3e}"


def test_host_gathered_shards_match_unsharded(ctx):
    case = cases.build(H=8, n_az=256, n_scans=3)
    full = _make(case, ctx, 0, 1)
    shards = [_make(case, ctx, r, 2) for r in range(2)]
    for p in shards:
        p.set_exchange_timing(True)
    assert [(p.h0, p.h1) for p in shards] == [(0, 4), (4, 8)]
    for k, s in enumerate(case["scans"]):
        full.stage_scan(0, s)
        full.run_scan(0, s, k)
        for p in shards:
            p.stage_scan(0, s)
            p.run_scan_local(0, s, k)
        recs = np.stack([p.partial() for p in shards])
        # only the rank holding hypothesis 0 contributes the map increment and the anchor
        from gcslam.pipeline import RECORD
        assert np.all(recs[1, RECORD["X0"][0]:] == 0.0)
        for p in shards:
            p.finish_scan(recs)
        ctx.sync()
        assert all(p.exchange_ms() >= 0.0 for p in shards)  # the record upload, timed on the stream
        ref = _state(full)
        st = [_state(p) for p in shards]
        for key in SHARED:
            assert np.array_equal(st[0][key], st[1][key]), f"scan{k} {key} differs between ranks"
            _rel_close(st[0][key], ref[key], 1e-12, f"scan{k} {key} vs unsharded")
        for key in ("L", "h", "X"):  # per-hypothesis results are independent of the sharding
            _rel_close(np.concatenate([st[0][key], st[1][key]]), ref[key], 1e-12, f"scan{k} {key}")


def test_rccl_single_rank_communicator(ctx):
    """ncclCommInitRank / ncclAllGather / ncclCommDestroy through gc_comm, then the pipeline's own
    all-gather path (a single-rank pipeline with a communicator gathers into a separate buffer):
    bit-identical to the pipeline without one."""
    import ctypes as C
    from gcslam import _abi
    from gcslam.pipeline import BatchedScanPipeline
    uid = BatchedScanPipeline.comm_unique_id()
    buf = (C.c_uint8 * _abi.GC_COMM_ID_BYTES).from_buffer_copy(uid)
    h = C.c_void_p()
    _abi.call("gc_comm_init", ctx.handle, 1, 0, C.addressof(buf), C.byref(h), ctx=ctx)
    x = np.arange(1000, dtype=np.float64) * 0.5
    ds, dr = _abi.DeviceArray.from_host(ctx, x), _abi.DeviceArray(ctx, 1000)
    _abi.call("gc_comm_allgather_f64", ctx.handle, h.value, ds.ptr, dr.ptr, 1000, ctx=ctx)
    ctx.sync()
    assert np.array_equal(dr.download(), x)
    ok = C.c_int32(-1)
    assert _abi.lib().gc_comm_healthy(h.value, C.byref(ok)) == _abi.GC_OK and ok.value == 1
    # after an abort the communicator reports unhealthy and every exchange is refused with the reason
    assert _abi.lib().gc_comm_abort(h.value) == _abi.GC_OK
    assert _abi.lib().gc_comm_healthy(h.value, C.byref(ok)) == _abi.GC_OK and ok.value == 0
    with pytest.raises(RuntimeError, match="refused.*aborted"):
        _abi.call("gc_comm_allgather_f64", ctx.handle, h.value, ds.ptr, dr.ptr, 1000, ctx=ctx)
    _abi.lib().gc_comm_destroy(h.value)

    case = cases.build(H=4, n_az=256, n_scans=2)
    plain, rccl = _make(case, ctx, 0, 1), _make(case, ctx, 0, 1)
    rccl.attach_comm(BatchedScanPipeline.comm_unique_id())
    for k, s in enumerate(case["scans"]):
        for p in (plain, rccl):
            p.stage_scan(0, s)
            p.run_scan(0, s, k)
    ctx.sync()
    a, b = _state(plain), _state(rccl)
    for key in a:
        assert np.array_equal(a[key], b[key]), key
    rccl.close()


def _gloo_rank(rank, world, port, outdir):
    sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from gcslam import _abi
    from oracle import cases as cs
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = _abi.Context(0)
    case = cs.build(H=6, n_az=256, n_scans=2)
    pipe = _make(case, ctx, rank, world)
    for k, s in enumerate(case["scans"]):
        pipe.stage_scan(0, s)
        pipe.run_scan_local(0, s, k)
        rec = torch.from_numpy(pipe.partial())
        out = [torch.empty_like(rec) for _ in range(world)]
        dist.all_gather(out, rec)
        pipe.finish_scan(torch.stack(out).numpy())
    ctx.sync()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **_state(pipe))
    pipe.close()
    dist.destroy_process_group()


def test_two_process_gloo_exchange_on_one_gpu(ctx, tmp_path):
    """Two processes (ranks 0, 1 of 3 / 3 hypotheses) on one GPU exchange their device partial
    records over gloo; both end bit-identical and match the unsharded pipeline."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    mp.spawn(_gloo_rank, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    st = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(2)]
    case = cases.build(H=6, n_az=256, n_scans=2)
    full = _make(case, ctx, 0, 1)
    for k, s in enumerate(case["scans"]):
        full.stage_scan(0, s)
        full.run_scan(0, s, k)
    ctx.sync()
    ref = _state(full)
    for key in SHARED:
        assert np.array_equal(st[0][key], st[1][key]), key
        _rel_close(st[0][key], ref[key], 1e-12, key)


def _dying_peer_rank(rank, world, port, outdir, timeout_s):
    """Rank 1 completes two scans, then dies (os._exit) before the third scan's exchange; rank 0
    must leave that exchange with an error within the bound, tear its pipeline down (bounded waits,
    a scan half still pending) and exit non-zero (backend_node.py:2205-2210: log and re-raise)."""
    import datetime
    import json
    import time
    sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from gcslam import _abi
    from oracle import cases as cs
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
    ctx = _abi.Context(0)
    ctx.set_wait_timeout(timeout_s)
    case = cs.build(H=6, n_az=256, n_scans=3)
    pipe = _make(case, ctx, rank, world)
    t_fail, err = None, None
    try:
        for k, s in enumerate(case["scans"]):
            pipe.stage_scan(0, s)
            pipe.run_scan_local(0, s, k)
            if rank == 1 and k == 2:
                os._exit(0)  # the peer dies mid-run: its third scan's local half done, no exchange
            rec = torch.from_numpy(pipe.partial())
            out = [torch.empty_like(rec) for _ in range(world)]
            t_fail = time.perf_counter()
            dist.all_gather(out, rec)
            pipe.finish_scan(torch.stack(out).numpy())
    except (RuntimeError, ValueError) as e:
        err = "%s: %s" % (type(e).__name__, str(e)[:300])
    waited = time.perf_counter() - t_fail if t_fail is not None else None
    t_close = time.perf_counter()
    pipe.close()  # the pending scan half is abandoned; destroy's waits are bounded
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump({"error": err, "waited_s": waited, "close_s": time.perf_counter() - t_close}, f)
    os._exit(3 if err else 0)


def test_peer_dying_mid_run_fails_the_survivor_within_bound(tmp_path):
    """Two processes on one GPU (ranks 0, 1 of 3 / 3 hypotheses, gloo exchange of the device partial
    records): rank 1 exits after its second full scan. Rank 0's third-scan exchange must fail (an
    error, not a hang) within the 20 s bound, its pipeline must tear down with the scan half pending,
    and it must exit non-zero."""
    import json
    import socket
    import time
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    bound = 20.0
    pctx = mp.get_context("spawn")
    procs = [pctx.Process(target=_dying_peer_rank, args=(r, 2, port, str(tmp_path), bound)) for r in range(2)]
    t0 = time.perf_counter()
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
            raise AssertionError("a rank is still running after 240 s")
    assert procs[1].exitcode == 0
    assert procs[0].exitcode == 3, procs[0].exitcode
    r0 = json.load(open(tmp_path / "rank0.json"))
    assert r0["error"] and r0["error"].startswith("RuntimeError"), r0
    assert r0["waited_s"] is not None and r0["waited_s"] < bound + 5.0, r0
    assert r0["close_s"] < 10.0, r0
    assert time.perf_counter() - t0 < 240.0
