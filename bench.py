#!/usr/bin/env python3
"""Benchmark: GC-SLAM v2 per-scan hot path on MI355X (BASELINE.json metric: LiDAR scans/s at
64k points x 256 hypotheses).

One "step" = one synthetic 64k-point scan through the batched per-scan pipeline for all H
hypotheses on this GPU (see DESIGN.md §Measurement for exactly which operators run inside
the step). Inputs are resident in HBM before the timed region; the timed region is bracketed
by a barrier + device synchronisation on both sides and the max over ranks is reported.

Extra legs (outside the timed region, same process):
  * roofline   — the contract decomposition BinSoftAssign + ScanBinMomentMatch over H
                 hypotheses (responsibilities materialised), timed per kernel with HIP events
                 on the library stream; achieved = algorithmic bytes / time.
  * cpu_baseline — the CPU oracle (NumPy restatement) on a bounded sample of the same
                 workload, rank 0 only, N=1 only.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
PROFILE_ROUNDS = ("r06", "r05", "r04", "r03", "r02", "r01")  # committed rocprofv3 summaries (profiles/<round>/), newest first


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50,
                    help="untimed steps first: the clocks ramp over the first ~30 ms of sustained f64 load")
    ap.add_argument("--prewarm-s", type=float, default=0.25,
                    help="untimed steps run for this many seconds before the --warmup steps, so a small W "
                         "still times the steady-state clocks (reported as prewarm_steps)")
    ap.add_argument("--hyps", type=int, default=256, help="total hypotheses per scan (strong scaling)")
    ap.add_argument("--n-az", type=int, default=4096, help="azimuth steps (x16 rings = points)")
    ap.add_argument("--scans", type=int, default=4, help="distinct resident scans cycled through")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-budget-s", type=float, default=30.0)
    ap.add_argument("--no-map", action="store_true", help="skip the C5 PrimitiveMap fuse leg")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 single-GPU pipeline leg")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the certs-on step and the per-stage timing scans after the timed region "
                         "(kernel traces whose last scans must be plain product scans)")
    ap.add_argument("--roofline-only", action="store_true",
                    help="run only the contract-pair roofline leg (PMC traffic passes, tools/pmc_traffic.sh)")
    ap.add_argument("--map-only", action="store_true",
                    help="run only the C5 PrimitiveMap fuse leg (PMC passes, tools/pmc_fuse.sh)")
    ap.add_argument("--c5-only", action="store_true", help="run only the C5 pipeline legs (PMC passes)")
    ap.add_argument("--c5-shard-only", action="store_true",
                    help="run only the C5 rank-shard leg (128 of 1024 hypotheses, with / without the map update)")
    ap.add_argument("--no-dropin", action="store_true", help="skip the per-operator drop-in leg")
    ap.add_argument("--dropin-only", action="store_true", help="run only the per-operator drop-in leg")
    ap.add_argument("--map-layout", choices=("packed", "fields"), default="packed",
                    help="device PrimitiveMap layout of the map legs (fields = the reference's per-field arrays)")
    ap.add_argument("--io-given", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--roofline-reps", type=int, default=10)
    ap.add_argument("--no-ingest", action="store_true",
                    help="stage the scans once before the timed region (round-2 methodology) instead of every step")
    ap.add_argument("--ingest-slots", type=int, default=INGEST_SLOTS,
                    help="scan slots in the ingest rotation (the slot staged at step k was last read by scan k - slots + 1)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch the ranks and exchange the communicator id, then exit (no GPU work)")
    ap.add_argument("--wait-timeout-s", type=float, default=120.0,
                    help="fail-fast bound (s) of every host wait: libgcslam's device waits (a timeout aborts "
                         "the RCCL communicator) and the gloo harness collectives; the bench then exits non-zero")
    ap.add_argument("--fail-rank", type=int, default=-1, help=argparse.SUPPRESS)  # test: this rank exits early
    return ap.parse_args()


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` without a torch.distributed.run environment: re-launch this script under
    torch.distributed.run with N ranks (one process per GPU) as a child process and return its exit
    code. Nothing in this parent process touches the GPU."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def dry_run(dist):
    """The rank launch and the communicator-id exchange without GPU work: rank 0 makes the RCCL
    unique id (a random token of the same size when no GPU is visible) and broadcasts it; rank 0
    prints every rank's view of (rank, world, id digest)."""
    import hashlib
    uid = None
    if dist.rank == 0:
        from gcslam import _abi
        try:
            from gcslam.pipeline import BatchedScanPipeline
            uid = BatchedScanPipeline.comm_unique_id() if _abi.device_count() > 0 else None
        except RuntimeError:
            uid = None
        uid = uid if uid is not None else os.urandom(128)
    if dist.world > 1:
        box = [uid]
        dist.td.broadcast_object_list(box, src=0)
        uid = box[0]
        views = [None] * dist.world
        dist.td.all_gather_object(views, (dist.rank, dist.world, hashlib.sha256(uid).hexdigest()))
    else:
        views = [(0, 1, hashlib.sha256(uid).hexdigest())]
    if dist.rank == 0:
        print(json.dumps({"dry_run": True, "n_ranks": dist.world, "ranks": views}), flush=True)


class Dist:
    """Host-side barrier / max-over-ranks for the bench harness (gloo); product collectives
    run in libgcslam over RCCL."""

    def __init__(self, n, timeout_s=120.0):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import datetime
            import torch.distributed as td
            # bounded: a rank whose peer died leaves its barrier / max with an error (gloo sees the closed
            # connection at once, or the timeout) instead of waiting out gloo's 30-minute default
            td.init_process_group("gloo", timeout=datetime.timedelta(seconds=timeout_s))
            self.td = td

    def barrier(self):
        if self.world > 1:
            self.td.barrier()

    def max(self, x: float) -> float:
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.td.all_reduce(t, op=self.td.ReduceOp.MAX)
        return float(t.item())


def workload_label(H_total: int, n: int, world: int) -> str:
    """The BASELINE.json config a run measures: C3 (64k x 256, 1 GPU), C4 (the same total over N
    ranks), C2 (H = 1); any other --hyps / --n-az is labelled by its own shape."""
    if n == 65536 and H_total == 256:
        return "C3" if world == 1 else "C4 (%d ranks)" % world
    if n == 65536 and H_total == 1:
        return "C2"
    if n == 65536 and 256 % H_total == 0:
        return "H=%d (one rank's shard of C4 at N=%d)" % (H_total, 256 // H_total)
    return "H=%d, %d points" % (H_total, n)


def pipe_partial_len(pipe):
    from gcslam.pipeline import partial_len
    return partial_len(pipe.B)


def bytes_soft_assign(n, B):
    return n * 24 + B * 24 + n * B * 8


def bytes_moment_match(n, B):
    return n * (24 + 72 + 8 + 8 + B * 8) + 24 + B * (1 + 3 + 9 + 3 + 9 + 1) * 8


INGEST_SLOTS = 3  # scan slots in the ingest rotation of the C3 step (--ingest-slots)


def warmup_map_record(ctx, _abi, scan, n, B, bins, origin):
    """Initial MapBinStats from one warm-up scan at the identity pose (zero pose covariance):
    the GPU bin statistics of the un-deskewed scan, pushed forward with R = I, t = 0."""
    from gcslam.constants import GC_TAU_SOFT_ASSIGN
    d = {k: _abi.DeviceArray.from_host(ctx, scan[k]) for k in ("points", "timestamps", "weights")}
    scal = _abi.DeviceArray(ctx, 8)
    _abi.call("gc_budget_stats", ctx.handle, d["weights"].ptr, n, n, scal.ptr, ctx=ctx)
    xi = _abi.DeviceArray.from_host(ctx, np.zeros((1, 6)))
    db = _abi.DeviceArray.from_host(ctx, bins)
    st, ce = _abi.DeviceArray(ctx, (1, B, 38)), _abi.DeviceArray(ctx, (1, 8))
    oa, op = _abi.f64p(origin)
    # a wide deskew window (t0 - 1000 s .. t1 + 1000 s) weights every point by the same ~0.987
    _abi.call("gc_scan_bins_fused", ctx.handle, 1, n, n, B, d["points"].ptr, d["timestamps"].ptr, d["weights"].ptr,
              scal.ptr, scan["scan_start"] - 1e3, scan["scan_end"] + 1e3, xi.ptr, db.ptr, GC_TAU_SOFT_ASSIGN, op,
              1e-12, 1e-12, st.ptr, ce.ptr, 0, ctx=ctx)
    s = st.download()[0]
    N, pb, Sp = s[:, 0], s[:, 13:16], s[:, 16:25].reshape(B, 3, 3)
    from gcslam.pipeline import map_record
    return map_record(s[:, 1:4], s[:, 4:13], N, N, N[:, None] * pb,
                      N[:, None, None] * (Sp + np.einsum("bi,bj->bij", pb, pb)))


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world_env}")
    dist = Dist(args.gpus, args.wait_timeout_s)
    if args.fail_rank == dist.rank:  # test of the fail-fast path: this rank dies before the id exchange
        os._exit(3)
    if args.dry_run:
        return dry_run(dist)
    from gcslam import _abi
    from gcslam.constants import GC_B_BINS, T_BASE_LIDAR
    from gcslam.ops.binning import create_fibonacci_atlas
    from gcslam.pipeline import BatchedScanPipeline, PipelineConfig, iw_meas_prior, iw_process_prior
    from gcslam.synth import make_hypotheses, make_scan

    ctx = _abi.Context(dist.local_rank)
    ctx.set_wait_timeout(args.wait_timeout_s)  # every device wait bounded; a timeout aborts the communicator
    H_total = args.hyps
    if args.map_only:
        print(json.dumps({"c5_map_fuse": map_fuse_leg(ctx, _abi, packed=args.map_layout == "packed")}), flush=True)
        return
    if args.dropin_only:
        print(json.dumps({"dropin": dropin_leg(ctx, _abi)}), flush=True)
        return
    if args.c5_only:
        print(json.dumps({"c5": c5_leg(ctx, _abi, args), "c5_dense": c5_leg(ctx, _abi, args, cap=131072)}),
              flush=True)
        return
    if args.c5_shard_only:
        print(json.dumps({"c5_shard": c5_shard_leg(ctx, _abi, args)}), flush=True)
        return
    if args.roofline_only:
        from gcslam.constants import GC_B_BINS, T_BASE_LIDAR
        from gcslam.ops.binning import create_fibonacci_atlas
        from gcslam.synth import make_scan
        s0 = make_scan(1, n_az=args.n_az)
        rng = np.random.default_rng(5)
        xi = np.zeros((H_total, 6)); xi[:, 0] = 0.1 + rng.normal(0, 0.005, H_total)
        xi[:, 5] = 0.03 + rng.normal(0, 0.002, H_total)
        d0 = {k: _abi.DeviceArray.from_host(ctx, s0[k]) for k in ("points", "timestamps", "weights")}
        dbins = _abi.DeviceArray.from_host(ctx, create_fibonacci_atlas(GC_B_BINS).dirs)
        r = roofline_leg(ctx, _abi, s0, d0, xi, dbins, GC_B_BINS, s0["points"].shape[0], H_total,
                         np.asarray(T_BASE_LIDAR[:3]), reps=args.roofline_reps)
        print(json.dumps({"roofline": r}), flush=True)
        return
    B = GC_B_BINS
    origin = np.asarray(T_BASE_LIDAR[:3])
    bins = create_fibonacci_atlas(B).dirs
    scans = [make_scan(k + 1, n_az=args.n_az) for k in range(args.scans)]
    n = scans[0]["points"].shape[0]
    pipe = BatchedScanPipeline(H_total, n, PipelineConfig(n_points_cap=n), rank=dist.rank,
                               world_size=dist.world, ctx=ctx)
    h0, h1 = pipe.h0, pipe.h1
    H = h1 - h0
    hy = make_hypotheses(H_total)
    pipe.set_beliefs(hy["X_anchor"][h0:h1], hy["z_lin"][h0:h1], hy["L"][h0:h1], hy["h"][h0:h1], hy["stamp"][h0:h1])
    pipe.set_weights(hy["weights"])
    if args.io_given:  # dev: IMU/odom-branch evidence given (isolates the branch's share of the step)
        from gcslam.synth import make_io_evidence
        pipe.set_io_evidence(*make_io_evidence(H))
    else:
        pipe.set_io_mode(True)  # IMU/odom branch evaluated on the device from each scan's odometry + IMU
    pipe.set_iw(*iw_process_prior(), *iw_meas_prior())
    pipe.set_map(warmup_map_record(ctx, _abi, make_scan(0, n_az=args.n_az), n, B, bins, origin))
    if dist.world > 1:
        uid = [pipe.comm_unique_id() if dist.rank == 0 else None]
        dist.td.broadcast_object_list(uid, src=0)
        pipe.attach_comm(uid[0])
    ingest = not args.no_ingest
    if not ingest:
        for k, s in enumerate(scans):
            pipe.stage_scan(k, s)

    count = [0]
    stage_s = [0.0, 0]  # host wall time inside stage_scan over the timed steps, and their count
    run_s = []          # host wall time of each timed run_scan call (enqueue + any wait for its slot)

    if ingest:
        pipe.stage_scan(0, scans[0])

    def step(timed=False):
        # with ingest, step k stages scan k+1 from host memory (pinned mirror + DMA on the copy
        # stream) into the next of three slots in rotation, then runs scan k: the copy of the next
        # scan overlaps this scan's compute (as a live node receives scan k+1 while it processes scan
        # k); every step stages exactly one scan. The slot it overwrites was read by scan k-2, whose
        # bins have normally published their completion already, so the DMA needs no ordering
        # event in the compute stream (gc_pipeline.cpp, done_word)
        k = count[0]
        sc = scans[k % len(scans)]
        if ingest:
            ts = time.perf_counter()
            pipe.stage_scan((k + 1) % args.ingest_slots, scans[(k + 1) % len(scans)])
            tr = time.perf_counter()
            pipe.run_scan(k % args.ingest_slots, sc, k)
            if timed:
                stage_s[0] += tr - ts
                stage_s[1] += 1
                run_s.append(time.perf_counter() - tr)
        else:
            pipe.run_scan(k % len(scans), sc, k)
        count[0] += 1

    # clock ramp: untimed steps for prewarm_s of sustained load (a 5-step W is ~7 ms, less than the
    # ~30 ms the clocks take to ramp under this f64 load), then the W warmup steps
    # (blocks of 10; every rank takes the same decision from the max over ranks, since each step
    # runs a collective when N > 1)
    t_pw = time.perf_counter()
    prewarm_steps = 0
    while args.prewarm_s > 0.0:
        for _ in range(10):
            step()
        prewarm_steps += 10
        ctx.sync()
        if dist.max(time.perf_counter() - t_pw) >= args.prewarm_s:
            break
    for _ in range(args.warmup):
        step()
    ctx.sync()
    dist.barrier()
    ctx.sync()
    pipe.host_stats(reset=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed=True)
    ctx.sync()
    dist.barrier()
    t1 = time.perf_counter()
    hs = pipe.host_stats(reset=True)
    elapsed = dist.max(t1 - t0)
    scans_per_s = args.steps / elapsed
    n_gpus = pipe.comm_size() if dist.world > 1 else 1  # the RCCL communicator's size
    exchange = None
    if dist.world > 1:
        # the per-scan all-gather's device time (HIP events around ncclAllGather on the pipeline
        # stream), untimed scans after the timed region: median over 20, max over ranks
        xs = []
        pipe.set_exchange_timing(True)  # events around the all-gather: off in the timed loop
        for _ in range(20):
            step()
            xs.append(pipe.exchange_ms())
        exchange = {"ms_median": dist.max(float(np.median(xs))), "record_bytes": 8 * pipe_partial_len(pipe),
                    "scans": len(xs), "op": "ncclAllGather (RCCL) of each rank's partial record"}

    out = {
        "metric": "LiDAR scans/sec (64k pts, 256 hypotheses) at 1/2/4/8 MI355X",
        "value": scans_per_s,
        "unit": "scans/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "prewarm_steps": prewarm_steps,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (VLP-16-like 16x%d ray-cast box room + 200 Hz IMU + wheel odometry, SURVEY §8d)"
                % args.n_az,
        "config": {"workload": "%s: one %d-point scan x %d hypotheses through the full batched pipeline "
                               "(a1-a16: budget, predict, IMU preint, deskew, soft-assign, moment-match, "
                               "Matrix-Fisher, planar, tempering, fusion, recompose, IW, map, anchor drift, "
                               "barycenter combine)" % (workload_label(H_total, n, dist.world), n, H_total),
                   "points": n, "hypotheses": H_total, "bins": B, "parallelism": "hypotheses/%d" % dist.world,
                   "ingest": ("every step stages one scan host -> HBM (pinned mirror + DMA on a copy stream): "
                              "step k stages scan k+1 while scan k computes (three slots in rotation)") if ingest else
                             "scans pre-staged in HBM before the timed region"},
    }
    if not args.no_extras:  # certs-on step time and per-stage device times (extras_leg)
        out_extra = extras_leg(pipe, ctx, dist, step)
    if exchange is not None:
        out["exchange"] = exchange
    if not args.no_extras:
        out.update(out_extra)
    ns = max(hs["scans"], 1.0)
    nst = max(hs["stages"], 1.0)
    out["host"] = {"scan_enqueue_ms": {"mean": hs["scan_enqueue_ms"] / ns, "max": hs["scan_enqueue_max_ms"]},
                   "scan_wait_ms": {"mean": hs["scan_wait_ms"] / ns, "max": hs["scan_wait_max_ms"]},
                   "stage_work_ms": {"mean": hs["stage_work_ms"] / nst, "max": hs["stage_work_max_ms"]},
                   "stage_wait_ms": {"mean": hs["stage_wait_ms"] / nst, "max": hs["stage_wait_max_ms"]},
                   "host_syncs": hs["host_syncs"], "h2d_bytes_per_scan": hs["h2d_bytes"] / ns,
                   "scans": hs["scans"],
                   "note": "libgcslam's own clock (gc_pipeline_host_stats): enqueue = the C entries' host work "
                           "(checks, launches, DMA issue), wait = polls / syncs on the device; the Python "
                           "run_scan_host_ms below also holds the ctypes overhead"}
    if ingest:
        out["ingest_host_ms_per_scan"] = 1e3 * stage_s[0] / max(stage_s[1], 1)
        out["run_scan_host_ms"] = {"mean": 1e3 * float(np.mean(run_s)), "max": 1e3 * float(np.max(run_s))}

    if dist.rank == 0 and not args.no_roofline:
        rng = np.random.default_rng(5)
        xi = np.zeros((H, 6)); xi[:, 0] = 0.1 + rng.normal(0, 0.005, H); xi[:, 5] = 0.03 + rng.normal(0, 0.002, H)
        d0 = {k: _abi.DeviceArray.from_host(ctx, scans[0][k]) for k in ("points", "timestamps", "weights")}
        dbins = _abi.DeviceArray.from_host(ctx, bins)
        out["roofline"] = roofline_leg(ctx, _abi, scans[0], d0, xi, dbins, B, n, H, origin, reps=args.roofline_reps)
    if dist.rank == 0 and not args.no_roofline:
        out["fused_roofline"] = fused_roofline_leg(ctx, _abi, scans[0], B, n, H, bins, origin)
    if dist.rank == 0 and not args.no_map:
        out["c5_map_fuse"] = map_fuse_leg(ctx, _abi, packed=args.map_layout == "packed")
    if dist.rank == 0 and dist.world == 1 and not args.no_dropin:
        out["dropin"] = dropin_leg(ctx, _abi)
    if dist.rank == 0 and dist.world == 1 and not args.no_c5:
        out["c5"] = c5_leg(ctx, _abi, args)
        out["c5_dense"] = c5_leg(ctx, _abi, args, cap=131072)
        out["c5_shard"] = c5_shard_leg(ctx, _abi, args)
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_leg(args.n_az, H_total, args.cpu_budget_s)
    if dist.rank == 0:
        print(json.dumps(out), flush=True)


def extras_leg(pipe, ctx, dist, step):
    """After the timed region: (1) the same step with the reference's per-call ConditioningCerts
    computed inside every scan (gc_pipeline_set_inscan_certs), 50 scans after 10 untimed, max over
    ranks; (2) the per-stage device time of the step (HIP events around each launch group; the
    events themselves cost the stream a few us each), median over 20 scans."""
    pipe.set_inscan_certs(True)
    for _ in range(10):
        step()
    ctx.sync()
    dist.barrier()
    tc0 = time.perf_counter()
    for _ in range(50):
        step()
    ctx.sync()
    dist.barrier()
    certs_ms = 1e3 * dist.max(time.perf_counter() - tc0) / 50
    pipe.set_inscan_certs(False)
    pipe.set_stage_timing(True)
    st_runs = []
    for _ in range(20):
        step()
        st_runs.append(pipe.stage_ms())
    pipe.set_stage_timing(False)
    stages = {k: float(np.median([r[k] for r in st_runs])) for k in st_runs[0]}
    return {"stages_ms": dict(stages, scans=len(st_runs), note="HIP events around each launch group, untimed scans"),
            "inscan_certs": {"ms_per_step": certs_ms, "scans": 50,
                             "note": "the same step with every hypothesis's predict and fusion ConditioningCert "
                                     "computed inside the scan (gc_pipeline_set_inscan_certs)"}}


def measured_traffic(H, n, B):
    """HBM bytes per launch of the contract pair from the committed rocprofv3 PMC summary
    (tools/pmc_traffic.sh; FETCH_SIZE doubled per the gfx950 correction, plus WRITE_SIZE), when it
    was collected at this exact shape; None otherwise."""
    for rnd in PROFILE_ROUNDS:  # the newest round's summary first
        f = os.path.join(ROOT, "profiles", rnd, "pmc_traffic.json")
        if os.path.exists(f):
            t = json.load(open(f))
            if (t.get("H"), t.get("n"), t.get("B")) == (H, n, B):
                return t
    return None


def roofline_leg(ctx, _abi, s, d, xi, dbins, B, n, H, origin, reps=10, warm=8, warm_s=0.3):
    """BinSoftAssign + ScanBinMomentMatch contract kernels over H hypotheses, HBM-bound."""
    from gcslam.constants import GC_TAU_SOFT_ASSIGN
    dxi = _abi.DeviceArray.from_host(ctx, xi)
    pts = _abi.DeviceArray(ctx, (H, n, 3)); w = _abi.DeviceArray(ctx, (H, n)); sw = _abi.DeviceArray(ctx, H)
    _abi.call("gc_deskew_constant_twist", ctx.handle, H, n, d["points"].ptr, d["timestamps"].ptr, d["weights"].ptr,
              s["scan_start"], s["scan_end"], dxi.ptr, pts.ptr, w.ptr, sw.ptr, ctx=ctx)
    dirs = _abi.DeviceArray(ctx, (H, n, 3))
    oa, op = _abi.f64p(origin)
    _abi.call("gc_point_directions", ctx.handle, H * n, pts.ptr, op, 1e-12, dirs.ptr, ctx=ctx)
    resp = _abi.DeviceArray(ctx, (H, n, B)); idx = _abi.DeviceArray(ctx, (H, n), np.int32)
    sac = _abi.DeviceArray(ctx, (H, 2))
    covs = _abi.DeviceArray(ctx, (H, n, 9)); covs.zero()
    lam = _abi.DeviceArray.from_host(ctx, np.ones((H, n)))
    st = _abi.DeviceArray(ctx, (H, B, 38)); ce = _abi.DeviceArray(ctx, (H, 8))
    # the pair back to back, reps times after warm untimed pairs (steady-state clocks, no host sync
    # between launches); one event before each kernel and one after the last, read after one sync
    def pair(r):
        _abi.call("gc_bin_soft_assign", ctx.handle, H, n, B, dirs.ptr, dbins.ptr, GC_TAU_SOFT_ASSIGN, resp.ptr,
                  idx.ptr, sac.ptr, ctx=ctx)
        ev[2 * r + 1].record()
        _abi.call("gc_scan_bin_moment_match", ctx.handle, H, n, B, pts.ptr, covs.ptr, w.ptr, resp.ptr, lam.ptr, op,
                  1e-12, 1e-12, st.ptr, ce.ptr, ctx=ctx)
        ev[2 * r + 2].record()

    ev = [_abi.Event(ctx) for _ in range(2 * reps + 1)]
    # warm pairs for at least warm_s of sustained load: the host-side set-up above leaves the GPU idle
    # long enough for its clocks to drop, and 8 pairs (~23 ms) did not always ramp them back (a box
    # measured the soft-assign at 1.52 ms here and 1.39 in the same command under rocprofv3)
    t_w, done = time.perf_counter(), 0
    while done < warm or time.perf_counter() - t_w < warm_s:
        for _ in range(4):
            _abi.call("gc_bin_soft_assign", ctx.handle, H, n, B, dirs.ptr, dbins.ptr, GC_TAU_SOFT_ASSIGN, resp.ptr,
                      idx.ptr, sac.ptr, ctx=ctx)
            _abi.call("gc_scan_bin_moment_match", ctx.handle, H, n, B, pts.ptr, covs.ptr, w.ptr, resp.ptr, lam.ptr,
                      op, 1e-12, 1e-12, st.ptr, ce.ptr, ctx=ctx)
        done += 4
        ctx.sync()
    ev[0].record()
    for r in range(reps):
        pair(r)
    ctx.sync()
    t_sa = [ev[2 * r].elapsed_ms(ev[2 * r + 1]) for r in range(reps)]
    t_mm = [ev[2 * r + 1].elapsed_ms(ev[2 * r + 2]) for r in range(reps)]
    ms_sa, ms_mm = float(np.mean(t_sa)), float(np.mean(t_mm))
    b_sa, b_mm = H * bytes_soft_assign(n, B), H * bytes_moment_match(n, B)
    ach = (b_sa + b_mm) / ((ms_sa + ms_mm) * 1e-3) / 1e9
    tr = measured_traffic(H, n, B)
    return {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "traffic": tr["pair_bytes"] if tr else None,
            "traffic_source": tr["source"] if tr else None,
            "kernel": "BinSoftAssign+ScanBinMomentMatch (k_soft_assign + k_moment_partials/k_bins_finalize)",
            "per_kernel": {"soft_assign": {"ms": ms_sa, "bytes": b_sa, "GB/s": b_sa / (ms_sa * 1e-3) / 1e9},
                           "moment_match": {"ms": ms_mm, "bytes": b_mm, "GB/s": b_mm / (ms_mm * 1e-3) / 1e9}},
            "hypotheses": H, "points": n, "bins": B}


FP64_PEAK_TFS = 78.6  # MI355X FP64 vector = FP64 matrix peak (16 lanes x FMA per SIMD-cycle, 256 CUs, 2.4 GHz)
FUSED_FLOP_PER_POINT_BIN = 76  # 5 (dot) + 1 (exp) + 2 (normalise) + 34 x 2 (moment FMAs)


def fused_roofline_leg(ctx, _abi, s, B, n, H, bins, origin, reps=10, warm=10):
    """The product's dominant kernel, k_bins_fused (a1->a4->a5->a6 fused, responsibilities in
    registers): FP64-issue-bound, so its roofline is flops against the FP64 peak. Timed with HIP
    events on the library stream around gc_scan_bins_fused (the fused kernel + its ~1 % finalize)."""
    from gcslam.constants import GC_TAU_SOFT_ASSIGN
    rng = np.random.default_rng(5)
    xi = np.zeros((H, 6)); xi[:, 0] = 0.1 + rng.normal(0, 0.005, H); xi[:, 5] = 0.03 + rng.normal(0, 0.002, H)
    d = {k: _abi.DeviceArray.from_host(ctx, s[k]) for k in ("points", "timestamps", "weights")}
    scal = _abi.DeviceArray(ctx, 8)
    _abi.call("gc_budget_stats", ctx.handle, d["weights"].ptr, n, n, scal.ptr, ctx=ctx)
    dx, db = _abi.DeviceArray.from_host(ctx, xi), _abi.DeviceArray.from_host(ctx, bins)
    st, ce = _abi.DeviceArray(ctx, (H, B, 38)), _abi.DeviceArray(ctx, (H, 8))
    oa, op = _abi.f64p(origin)
    def launch():
        _abi.call("gc_scan_bins_fused", ctx.handle, H, n, n, B, d["points"].ptr, d["timestamps"].ptr,
                  d["weights"].ptr, scal.ptr, s["scan_start"], s["scan_end"], dx.ptr, db.ptr, GC_TAU_SOFT_ASSIGN, op,
                  1e-12, 1e-12, st.ptr, ce.ptr, 0, ctx=ctx)

    for _ in range(warm):  # back to back (steady-state clocks), then reps launches between two events
        launch()
    ev = [_abi.Event(ctx) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        launch()
    ev[1].record()
    ctx.sync()
    ms = ev[0].elapsed_ms(ev[1]) / reps
    flop = float(FUSED_FLOP_PER_POINT_BIN) * n * B * H
    ach = flop / (ms * 1e-3) / 1e12
    return {"bound": "fp64", "achieved": ach, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s", "frac": ach / FP64_PEAK_TFS,
            "ms": ms, "flop": flop, "flop_per_point_bin": FUSED_FLOP_PER_POINT_BIN,
            "kernel": "k_bins_fused + k_bins_finalize (gc_scan_bins_fused)", "hypotheses": H, "points": n, "bins": B}


def c5_leg(ctx, _abi, args, H=1024, n_az=8192, cap=65536, steps=10, warmup=5, m_slots=1 << 20, voxel=0.1,
           map_update=True):
    """C5 on one GPU: 131,072-point scans budgeted to 65,536 (stride 2) x 1024
    hypotheses through the full batched pipeline, each scan staged from host memory and fused into
    a resident 1M-slot PrimitiveMap by the in-scan map update (csrc/gc_scanmap.hip). BASELINE.json
    quotes C5 on 8 GPUs; this is one GPU's whole-job throughput at the full 1024 hypotheses.
    H=128: one rank's shard of C5 on 8 GPUs; map_update=False times it without the update (the
    non-owner ranks: only hypothesis 0's rank runs it, include/gcslam.h GC_SMAP_OWNER)."""
    from gcslam.constants import GC_B_BINS, T_BASE_LIDAR
    from gcslam.ops.binning import create_fibonacci_atlas
    from gcslam.pipeline import BatchedScanPipeline, PipelineConfig, iw_meas_prior, iw_process_prior
    from gcslam.synth import make_hypotheses, make_scan
    B = GC_B_BINS
    scans = [make_scan(k + 1, n_az=n_az) for k in range(2)]
    n_in = scans[0]["points"].shape[0]
    pipe = BatchedScanPipeline(H, n_in, PipelineConfig(n_points_cap=cap), ctx=ctx)
    hy = make_hypotheses(H)
    pipe.set_beliefs(hy["X_anchor"], hy["z_lin"], hy["L"], hy["h"], hy["stamp"])
    pipe.set_weights(hy["weights"])
    pipe.set_io_mode(True)
    pipe.set_iw(*iw_process_prior(), *iw_meas_prior())
    pipe.set_map(warmup_map_record(ctx, _abi, make_scan(0, n_az=n_az), n_in, B, create_fibonacci_atlas(B).dirs,
                                   np.asarray(T_BASE_LIDAR[:3])))
    if map_update:
        dm = primitive_map_1m(ctx, m_slots)
        pipe.attach_primitive_map(dm, voxel)  # the in-scan map update runs inside every timed scan

    pipe.stage_scan(0, scans[0])

    def step(i):  # double-buffered ingest, as the C3 step
        pipe.stage_scan((i + 1) % 2, scans[(i + 1) % 2])
        pipe.run_scan(i % 2, scans[i % 2], i)

    for i in range(warmup):
        step(i)
    ctx.sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    ctx.sync()
    dt = (time.perf_counter() - t0) / steps
    touched = pipe.scan_map_count() if map_update else 0
    pipe.close()
    stride = -(-n_in // cap)
    upd = ("the in-scan PrimitiveMap update (%d rows into a %d-slot map, voxel %.2f m)" % (cap, m_slots, voxel)
           if map_update else "no map update (a non-owner rank)")
    return {"workload": "C5 shape on 1 GPU: %d-point scans (staged every step), budget cap %d (%s), %d "
                        "hypotheses, full pipeline + %s" % (n_in, cap, "dense: every point" if stride == 1 else
                                                            "stride %d" % stride, H, upd),
            "ms_per_scan": 1e3 * dt, "scans_per_s": 1.0 / dt, "steps": steps, "warmup": warmup,
            "map_slots_touched_last_scan": touched}


def c5_shard_leg(ctx, _abi, args, H=128):
    """One rank's shard of C5 on 8 GPUs (1024 / 8 = 128 hypotheses, 131,072-point scans, stride 2): the
    owner rank's step (hypothesis 0's rank: the in-scan map update on its side stream) and a non-owner
    rank's (no update, GC_SMAP_OWNER). The exchange is not in it (no communicator on one GPU)."""
    own = c5_leg(ctx, _abi, args, H=H, steps=20, warmup=10)
    other = c5_leg(ctx, _abi, args, H=H, steps=20, warmup=10, map_update=False)
    return {"hypotheses": H, "of": 1024, "owner_ms_per_scan": own["ms_per_scan"],
            "non_owner_ms_per_scan": other["ms_per_scan"],
            "update_cost_ms": own["ms_per_scan"] - other["ms_per_scan"],
            "map_slots_touched_last_scan": own["map_slots_touched_last_scan"],
            "note": "the scan rate of C5 on 8 GPUs is bounded by the slower of the two (max over ranks) plus the "
                    "per-scan all-gather"}


def dropin_leg(ctx, _abi, K=4, cap=8192, n_az=4096, warm=3, scans=10):
    """The reference node's own configuration through the per-operator drop-ins (gcslam.dropin_node):
    K_HYP = 4 hypotheses, N_POINTS_CAP = 8192 (common/constants.py:62-64) on the 65,536-point synthetic
    scan, each hypothesis's operator chain (budget, predict, windows, preintegration, deskew, directions,
    soft-assign, moment match, Matrix-Fisher, planar, excitation, fusion, recompose, IW statistics, anchor
    drift) with its point arrays and responsibilities device-resident, then the barycenter and the IW
    applies (backend_node.py:2036-2119). ms per scan over `scans` scans after `warm`; the arena's hipMalloc /
    hipFree count over the timed scans (0: every buffer reused)."""
    import gc as _gc
    from gcslam.belief import BeliefGaussianInfo
    from gcslam.constants import GC_B_BINS, GC_CHART_ID, T_BASE_LIDAR
    from gcslam.dropin_node import BinMap, DropinNode, IOGiven
    from gcslam.ops import MeasurementNoiseIWState, ProcessNoiseIWState
    from gcslam.ops.binning import create_fibonacci_atlas
    from gcslam.pipeline import BatchedScanPipeline, PipelineConfig, iw_meas_prior, iw_process_prior
    from gcslam.synth import make_hypotheses, make_io_evidence, make_scan
    B = GC_B_BINS
    bins = create_fibonacci_atlas(B).dirs
    sc = [make_scan(k + 1, n_az=n_az) for k in range(2)]
    n = sc[0]["points"].shape[0]
    rec = warmup_map_record(ctx, _abi, make_scan(0, n_az=n_az), n, B, bins, np.asarray(T_BASE_LIDAR[:3]))
    # the map-derived statistics by the device's k_map_derive (a one-hypothesis pipeline used as the tool)
    p1 = BatchedScanPipeline(1, n, PipelineConfig(n_points_cap=cap), ctx=ctx)
    p1.set_map(rec)
    mp = p1.get_map()
    p1.close()
    hy = make_hypotheses(K)
    Lio, hio, cio = make_io_evidence(K)
    nuP, PsiP = iw_process_prior()
    nuM, PsiM = iw_meas_prior()
    pn = ProcessNoiseIWState(np.asarray(nuP, np.float64).reshape(7), np.asarray(PsiP, np.float64).reshape(7, 6, 6))
    mn = MeasurementNoiseIWState(np.asarray(nuM, np.float64).reshape(3), np.asarray(PsiM, np.float64).reshape(3, 3, 3))
    from gcslam.ops import process_noise_state_to_Q_jax
    beliefs = [BeliefGaussianInfo(GC_CHART_ID, "initial", hy["X_anchor"][i], hy["stamp"][i], hy["z_lin"][i], hy["L"][i],
                                  hy["h"][i]) for i in range(K)]
    node = DropinNode(beliefs, hy["weights"], bins, BinMap(mp["map"], mp["derived"]), process_noise_state_to_Q_jax(pn),
                      pn, mn, cap, ctx=ctx)
    ios = [IOGiven(Lio[i], hio[i], cio[i]) for i in range(K)]
    for k in range(warm):
        node.process_scan(sc[k % 2], ios)
    ctx.sync()
    _gc.collect()
    a0 = ctx.alloc_stats()
    t0 = time.perf_counter()
    for k in range(scans):
        node.process_scan(sc[k % 2], ios)
    ctx.sync()
    dt = (time.perf_counter() - t0) / scans
    _gc.collect()
    a1 = ctx.alloc_stats()
    return {"workload": "reference node configuration through the per-operator drop-ins: K_HYP = %d, N_POINTS_CAP = "
                        "%d (stride %d from %d points), legacy bin-path operator chain per hypothesis + barycenter + "
                        "IW applies (gcslam.dropin_node)" % (K, cap, -(-n // cap), n),
            "ms_per_scan": 1e3 * dt, "scans_per_s": 1.0 / dt, "scans": scans, "warmup": warm,
            "hip_mallocs": a1["hip_mallocs"] - a0["hip_mallocs"], "hip_frees": a1["hip_frees"] - a0["hip_frees"],
            "arena_reuses": a1["reuses"] - a0["reuses"],
            "note": "host-driven (one ctypes call + the certificate download per operator, as the reference's "
                    "wrappers sync per cert); the reference publishes ~1-2 s per scan on its JAX GPU path "
                    "(backend_node.py:1142, SURVEY §6)"}


def primitive_map_1m(ctx, M, seed=20261015):
    """A resident M-slot PrimitiveMap (random SPD Λ with eigenvalues 10..1e4, θ, 3-lobe η, w in (0, 1])."""
    from gcslam.primitive_map import DevicePrimitiveMap
    rng = np.random.default_rng(seed)
    Q, _ = np.linalg.qr(rng.normal(size=(M, 3, 3)))
    dm = DevicePrimitiveMap(1, M, ctx=ctx)
    dm.upload(Lambdas=np.einsum("nij,nj,nkj->nik", Q, 10.0 ** rng.uniform(1, 4, (M, 3)), Q),
              thetas=rng.normal(size=(M, 3)), etas=rng.normal(size=(M, 3, 3)), weights=rng.uniform(1e-3, 1.0, M))
    return dm


def map_fuse_leg(ctx, _abi, m_slots=1 << 20, rows=1 << 17, reps=5, packed=True):
    """C5 map update: 1,048,576-slot PrimitiveMap (random SPD Λ with eigenvalues
    10..1e4, θ, 3-lobe η, w in (0, 1]) and 131,072 measurement rows pushed to the world frame and
    fused (transform_gaussian_to_world + primitive_map_fuse, colour tracking on)."""
    from gcslam.primitive_map import DeviceFuseBatch, DevicePrimitiveMap, fuse_device
    rng = np.random.default_rng(20261015)
    M, K, Lb = m_slots, rows, 3

    def spd(n):
        Q, _ = np.linalg.qr(rng.normal(size=(n, 3, 3)))
        return np.einsum("nij,nj,nkj->nik", Q, 10.0 ** rng.uniform(1, 4, (n, 3)), Q)

    dm = DevicePrimitiveMap(1, M, ctx=ctx, packed=packed)
    dm.upload(Lambdas=spd(M), thetas=rng.normal(size=(M, 3)), etas=rng.normal(size=(M, Lb, 3)),
              weights=rng.uniform(1e-3, 1.0, M))
    slots = rng.integers(0, M, K)
    batch = DeviceFuseBatch(ctx, slots, spd(K), rng.normal(size=(K, 3)), rng.normal(size=(K, Lb, 3)),
                            rng.uniform(0, 1, K), rng.uniform(0, 1, K), rng.uniform(0, 1, K) > 0.05,
                            rng.uniform(0, 1, (K, 3)), np.ones(K, np.int32))
    pose = np.array([1.0, -2.0, 0.0, 0.01, -0.02, 0.7])
    n_unique = fuse_device(dm, batch, 0.0, 0, pose)  # warm (and the touched-slot count)
    ev = [_abi.Event(ctx) for _ in range(2)]
    ev[0].record()
    for r in range(reps):
        fuse_device(dm, batch, float(r + 1), r + 1, pose, count=False)
    ev[1].record()
    ctx.sync()
    ms = ev[0].elapsed_ms(ev[1]) / reps
    row_b = 4 + 72 + 24 + 72 + 8 + 8 + 1 + 24 + 4
    slot_rmw = 2 * (72 + 24 + 72 + 8 + 8 + 24 + 8 + 24 + 8)   # core 176 B + stamps/seqs + cam/lidar/accum/denom
    # the colour estimate: the map's colours are current after the first fuse, so only the touched
    # slots' rgb / colors are rewritten (the same map as the reference's all-slot recompute)
    colour = n_unique * (24 + 24)
    b = K * row_b + n_unique * slot_rmw + colour
    # round 2's accounting: the reference's all-slot colour pass (every slot's cam/denom/accum read,
    # rgb/colors written) counted as algorithmic bytes
    b_all = K * row_b + n_unique * slot_rmw + M * (8 + 8 + 24 + 24 + 24)
    return {"slots": M, "rows": K, "distinct_slots": n_unique, "ms": ms, "bytes": b,
            "GB/s": b / (ms * 1e-3) / 1e9, "bytes_all_slot_colour": b_all,
            "GB/s_all_slot_colour": b_all / (ms * 1e-3) / 1e9, "layout": "packed" if packed else "fields",
            "kernel": "k_fuse_runs + k_fuse_apply_blk (per-block register sort, run hash of the touched slots; the sort block's rows staged in LDS; colour estimate of the touched slots)"}


def cpu_info():
    """os.cpu_count(), the affinity count, the cgroup CPU quota (cpu.max, if any) and the model."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(float(q) / float(per)))
    except (OSError, ValueError):
        pass
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return dict(cpu_count=os.cpu_count(), affinity=aff, cgroup_quota=quota, model=model)


_CPU = {}


def _cpu_init(n_az, H_total):
    """Per-process oracle inputs of the C3 scan (spawned pool workers build their own copy)."""
    sys.path.insert(0, ROOT)
    from threadpoolctl import threadpool_limits
    from oracle import cases, gc_oracle as O
    _CPU["limits"] = threadpool_limits(limits=1)
    case = cases.build(H=H_total, n_az=n_az, n_scans=1, io="computed")
    st = case["state"]
    _CPU.update(case=case, scan=cases.scan_input(case["scans"][0]), Q=O.iw_process_Q(st.nu_proc, st.Psi_proc),
                Sga=(O.iw_meas_mode(st.nu_meas, st.Psi_meas, 0), O.iw_meas_mode(st.nu_meas, st.Psi_meas, 1)),
                md=O.map_derived(st.map))


def _cpu_hyp(k):
    """One hypothesis through a1-a15 (+ the IMU/odom branch) in the oracle."""
    from oracle import gc_oracle as O
    c = _CPU["case"]
    st = c["state"]
    r = O.scan_hypothesis(st.beliefs[k], _CPU["scan"], _CPU["Q"], None, st.map, _CPU["md"], c["bins"], c["cfg"],
                          _CPU["Sga"])
    return (r["belief"], r["dPsi_proc"], r["dPsi_meas"], r["map_inc"] if k == 0 else None)


def _cpu_combine(outs, st):
    """a16 barycenter + IW apply + map update of one scan (backend_node.py:2085-2119)."""
    from oracle import gc_oracle as O
    H = len(outs)
    w = st.weights
    comb = O.hypothesis_barycenter(np.stack([o[0].L for o in outs]), np.stack([o[0].h for o in outs]),
                                   np.stack([o[0].z_lin for o in outs]), w, 0.01 / H)
    aP = sum(w[i] * outs[i][1] for i in range(H))
    aM = sum(w[i] * outs[i][2] for i in range(H))
    O.iw_process_apply(st.nu_proc, st.Psi_proc, aP, np.full(7, w.sum()))
    O.iw_meas_apply(st.nu_meas, st.Psi_meas, aM, w.sum() * np.array([1.0, 1.0, 0.0]))
    O.map_forget_and_add(st.map, outs[0][3])
    return comb


def cpu_leg(n_az, H_total, budget_s):
    """CPU baseline: the oracle (NumPy restatement of the reference path) on the
    same C3 scan, both legs of the plan, on this host's cores:
      (i)  one process, BLAS threads = the usable cores: per-hypothesis a1-a15 timed as the median
           of 20 hypotheses after 3 warm-ups, plus one timed a16 combine + IW apply + map update
           over all H; scan time = H x median + combine;
      (ii) multiprocessing.Pool(usable cores) over the hypotheses (1 BLAS thread per worker): whole
           scans (all H hypotheses, then the combine in the parent), median of the scans that fit
           the budget after one warm-up scan.
    Usable cores = min(affinity, cgroup quota)."""
    import multiprocessing as mproc
    import statistics
    from threadpoolctl import threadpool_limits
    info = cpu_info()
    cores = min(info["affinity"], info["cgroup_quota"] or info["affinity"])
    _cpu_init(n_az, H_total)
    st = _CPU["case"]["state"]
    # leg (i)
    with threadpool_limits(limits=cores):
        for k in range(3):
            _cpu_hyp(k % H_total)
        ts, outs = [], []
        for k in range(20):
            t0 = time.perf_counter()
            outs.append(_cpu_hyp(k % H_total))
            ts.append(time.perf_counter() - t0)
        t_hyp = statistics.median(ts)
        full = [outs[0]] + [outs[1 + (k % 19)] for k in range(H_total - 1)]
        t0 = time.perf_counter()
        _cpu_combine(full, st)
        t_comb = time.perf_counter() - t0
    leg1 = {"scans_per_s": 1.0 / (H_total * t_hyp + t_comb), "median_hyp_ms": 1e3 * t_hyp,
            "combine_ms": 1e3 * t_comb, "blas_threads": cores,
            "sample": "20 hypotheses after 3 warm-ups (median) x %d + one combine/IW/map over %d" % (H_total, H_total)}
    # leg (ii)
    pctx = mproc.get_context("spawn")  # fresh interpreters: nothing of this process's GPU state
    scans = []
    with pctx.Pool(cores, initializer=_cpu_init, initargs=(n_az, H_total)) as pool:
        pool.map(_cpu_hyp, [k % H_total for k in range(cores)])  # workers built and warm
        t_start = time.perf_counter()
        n = 0
        while n < 6 and (n < 2 or time.perf_counter() - t_start < budget_s):
            t0 = time.perf_counter()
            outs = pool.map(_cpu_hyp, range(H_total), chunksize=max(1, H_total // (4 * cores)))
            _cpu_combine(outs, st)
            dt = time.perf_counter() - t0
            if n > 0:  # the first scan is the warm-up
                scans.append(dt)
            n += 1
    t_scan = statistics.median(scans)
    leg2 = {"scans_per_s": 1.0 / t_scan, "median_scan_s": t_scan, "workers": cores,
            "sample": "%d whole %d-hypothesis scans after 1 warm-up (median)" % (len(scans), H_total)}
    best = max(leg1["scans_per_s"], leg2["scans_per_s"])
    return {"value": best, "unit": "scans/s", "cores": cores, "kind": "port",
            "sample": "oracle (NumPy restatement) on the %s scan, %d points x %d hypotheses, a1-a16 incl. the "
                      "IMU/odom branch, combine, IW apply and map update; value = the faster of leg (i) %s and "
                      "leg (ii) Pool(%d) %s" % (workload_label(H_total, _CPU["case"]["n"], 1).split(" ")[0].rstrip(","),
                                                _CPU["case"]["n"], H_total, leg1["sample"], cores, leg2["sample"]),
            "legs": {"single_process": leg1, "pool": leg2}, **info}


if __name__ == "__main__":
    try:
        main()
    except Exception as e:  # fail fast (backend_node.py:2205-2210: log and re-raise): a non-zero exit
        print(json.dumps({"error": "%s: %s" % (type(e).__name__, e), "rank": os.environ.get("RANK", "0")}),
              file=sys.stderr, flush=True)
        raise
