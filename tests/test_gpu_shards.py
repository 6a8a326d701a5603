"""The multi-GPU configurations' per-rank geometries on one GPU (backend_node.py:2036-2119).

C4 (256 hypotheses over 8 GPUs) and C5 (1024 over 8) run every rank's shard as its own
BatchedScanPipeline on this device: 8 x 32 of 256 at 65,536 points, and 8 x 128 of 1024 at 131,072
points budgeted to 65,536 (stride 2), with the IMU/odom branch computed, so k_bins_io runs the
task tiers of a 32- / 128-hypothesis shard. Each scan is run_scan_local on every shard, the 8
partial records stacked on the host in rank order, then finish_scan(records) on every shard: the
G = 8 rank-ordered reduction of k_combine_final that the RCCL all-gather feeds on the 8-GPU node.

Bars:
  * the combined belief, IW state, Q and map are bit-identical on all 8 shards;
  * against the unsharded pipeline run beside them: with the shards' chunk geometry sized as
    for the full hypothesis count (geometry_hyps = H) every per-hypothesis result of the first scan
    is bit-identical, the shared state within 1e-12 relative (the 8 shard sums associate
    differently from one) and so, through it, every later scan's per-hypothesis results;
    at the production geometry (each shard sized for its own 32 / 128 hypotheses, as the bench
    runs) the per-hypothesis sums run in another order, so the bars are the oracle's;
  * sampled hypotheses on both sides of every shard boundary tested (0, 31, 32, 255 for C4;
    0, 127, 128, 1023 for C5) against the oracle at the bars of test_gpu_configs.py, and the
    couplings (barycenter, IW apply, map) from the shards' per-hypothesis outputs of ALL hypotheses.
"""

import numpy as np
import pytest

from oracle import cases
from test_gpu_configs import _FAILS, _pipeline, _run_and_compare

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _report():
    _FAILS.clear()
    yield
    assert not _FAILS, "\n".join(_FAILS[:60])


def _rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


class ShardSet:
    """world_size shards of one hypothesis set on this device, driven in lockstep with the host
    gather standing in for RCCL; exposes the BatchedScanPipeline surface _run_and_compare uses
    (per-hypothesis arrays concatenated in rank order, shared state from rank 0)."""

    SHARED = ("comb_L", "comb_h", "comb_z", "comb_X", "nu_proc", "Psi_proc", "nu_meas", "Psi_meas", "Q", "map",
              "map_der")

    def __init__(self, case, ctx, H, cap, world, geometry_hyps=0, full=None, exact_vs_full=False):
        self.shards = [_pipeline(case, ctx, H, cap, True, rank=r, world=world, geometry_hyps=geometry_hyps)
                       for r in range(world)]
        self.full, self.exact = full, exact_vs_full
        self.k = 0
        self.report = []

    @staticmethod
    def _shared(p):
        c, iw, mp = p.combined(), p.get_iw(), p.get_map()
        return dict(comb_L=c["L"], comb_h=c["h"], comb_z=c["z_lin"], comb_X=c["X_anchor"], nu_proc=iw["nu_proc"],
                    Psi_proc=iw["Psi_proc"], nu_meas=iw["nu_meas"], Psi_meas=iw["Psi_meas"], Q=iw["Q"],
                    map=mp["map"], map_der=mp["derived"])

    def stage_scan(self, slot, s):
        for p in self.shards:
            p.stage_scan(slot, s)
        if self.full is not None:
            self.full.stage_scan(slot, s)

    def run_scan(self, slot, s, k):
        for p in self.shards:
            p.run_scan_local(slot, s, k)
        recs = np.stack([p.partial() for p in self.shards])
        for p in self.shards:
            p.finish_scan(recs)
        if self.full is not None:
            self.full.run_scan(slot, s, k)
        self._check(k)
        self.k += 1

    def _check(self, k):
        st = [self._shared(p) for p in self.shards]
        for r in range(1, len(st)):
            for key in self.SHARED:
                if not np.array_equal(st[0][key], st[r][key]):
                    _FAILS.append(f"scan{k} {key}: rank {r} differs from rank 0")
        if self.full is None:
            return
        ref = self._shared(self.full)
        for key in self.SHARED:
            e = _rel(st[0][key], ref[key])
            self.report.append((k, key, e))
            if self.exact and not e <= 1e-12:
                _FAILS.append(f"scan{k} {key} vs unsharded: {e:.3e} relative (bar 1e-12)")
        b, bf = self.get_beliefs(), self.full.get_beliefs()
        # bit-identical per hypothesis on the first scan; from the second on, the shared state the
        # scan starts from (Q from the IW state, the map) carries the 1e-16 of the cross-shard sums
        first = self.k == 0
        for key in ("X_anchor", "z_lin", "L", "h"):
            e = _rel(b[key], bf[key])
            self.report.append((k, key, e))
            if self.exact and first and not np.array_equal(b[key], bf[key]):
                _FAILS.append(f"scan{k} per-hypothesis {key} not bit-identical to the unsharded pipeline")
            elif self.exact and not e <= 1e-12:
                _FAILS.append(f"scan{k} per-hypothesis {key} vs unsharded: {e:.3e} relative (bar 1e-12)")
        if self.exact and first:
            for a, c in zip(self.bin_stats(), self.full.bin_stats()):
                if not np.array_equal(a, c):
                    _FAILS.append(f"scan{k} bin statistics not bit-identical to the unsharded pipeline")

    def _cat(self, f):
        outs = [f(p) for p in self.shards]
        if isinstance(outs[0], dict):
            return {k: np.concatenate([o[k] for o in outs]) for k in outs[0]}
        if isinstance(outs[0], tuple):
            return tuple(np.concatenate([o[i] for o in outs]) for i in range(len(outs[0])))
        return np.concatenate(outs)

    def get_beliefs(self):
        return self._cat(lambda p: p.get_beliefs())

    def hyp_diag(self):
        return self._cat(lambda p: p.hyp_diag())

    def hyp_conditioning(self):
        return self._cat(lambda p: p.hyp_conditioning())

    def bin_stats(self):
        return self._cat(lambda p: p.bin_stats())

    def hyp_stats(self):
        return self._cat(lambda p: p.hyp_stats())

    def projection_certs(self):
        outs = [p.projection_certs() for p in self.shards]
        d = dict(outs[0])  # the scan-level certificates: every rank's combine forms the same ones
        for k in ("bins", "mf", "planar"):
            d[k] = np.concatenate([o[k] for o in outs])
        return d

    def get_iw(self):
        return self.shards[0].get_iw()

    def get_map(self):
        return self.shards[0].get_map()

    def combined(self):
        return self.shards[0].combined()


def _shard_run(ctx, case, H, cap, world, sample, n_scans, geometry_hyps, exact):
    full = _pipeline(case, ctx, H, cap, True)
    view = ShardSet(case, ctx, H, cap, world, geometry_hyps=geometry_hyps, full=full, exact_vs_full=exact)
    assert [(p.h0, p.h1) for p in view.shards] == [(H * r // world, H * (r + 1) // world) for r in range(world)]
    _run_and_compare(ctx, case, H, cap, sample, n_scans, True, pipe=view)
    worst = {}
    for k, key, e in view.report:
        worst[key] = max(worst.get(key, 0.0), e)
    print("max relative difference vs the unsharded pipeline:", {k: f"{v:.2e}" for k, v in worst.items()})
    for p in view.shards + [full]:
        p.close()


def test_c4_rank_shards_production_geometry(ctx):
    """C4: 8 shards x 32 of 256 hypotheses at 65,536 points (each shard's own k_bins_io tiers),
    two scans (the second with the process-IW update and the cached posterior factorisation)."""
    case = cases.build(H=256, n_az=4096, n_scans=2, io="computed")
    _shard_run(ctx, case, 256, case["n"], 8, [0, 31, 32, 255], 2, 0, False)


def test_c4_rank_shards_bit_identical_per_hypothesis(ctx):
    """C4 with geometry_hyps = 256 on every shard: each hypothesis's points are summed in the
    unsharded order, so every per-hypothesis result equals the unsharded pipeline's bit for bit."""
    case = cases.build(H=256, n_az=4096, n_scans=2, io="computed")
    _shard_run(ctx, case, 256, case["n"], 8, [0, 255], 2, 256, True)


def test_c5_rank_shards_production_geometry(ctx):
    """C5: 8 shards x 128 of 1024 hypotheses, 131,072-point scans budgeted to 65,536 (stride 2)."""
    case = cases.build(H=1024, n_az=8192, n_scans=1, io="computed", cap=65536)
    _shard_run(ctx, case, 1024, 65536, 8, [0, 127, 128, 1023], 1, 0, False)
