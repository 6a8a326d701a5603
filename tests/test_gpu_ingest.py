"""Per-scan ingest on the pipeline's copy stream (backend_node.py:1679-1690) and the state lock
between the two halves of a scan.

Staging copies the caller's arrays into the slot's pinned mirror before returning and DMAs them
into HBM on a copy stream, ordered after the last scan that read the slot; scan_local waits for
the slot's copy. These tests drive the orders a live loop produces — the next scan staged while
the current one runs, a slot restaged while the scan that reads it is still queued, the caller's
arrays overwritten as soon as staging returns — and require the results to be bit-identical to
synchronous staging."""

import numpy as np
import pytest

from oracle import cases
from test_gpu_configs import _pipeline

pytestmark = pytest.mark.gpu


def _state(p):
    b, c, iw, mp = p.get_beliefs(), p.combined(), p.get_iw(), p.get_map()
    return dict(L=b["L"], h=b["h"], X=b["X_anchor"], z=b["z_lin"], comb_L=c["L"], comb_h=c["h"], Psi=iw["Psi_proc"],
                Psim=iw["Psi_meas"], Q=iw["Q"], map=mp["map"])


def _assert_same(a, b):
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def _scrambled_copy(s):
    """A copy of the scan whose arrays the test overwrites right after staging."""
    return {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in s.items()}


def _scramble(s):
    for v in s.values():
        if isinstance(v, np.ndarray) and v.dtype.kind == "f":
            v[...] = np.nan


def test_stage_ahead_two_slots_matches_synchronous(ctx):
    case = cases.build(H=16, n_az=1024, n_scans=5, io="computed")
    ref = _pipeline(case, ctx, 16, case["n"], True)
    for k, s in enumerate(case["scans"]):
        ref.stage_scan(0, s)
        ref.run_scan(0, s, k)
        ctx.sync()
    want = _state(ref)
    p = _pipeline(case, ctx, 16, case["n"], True)
    scans = case["scans"]
    c0 = _scrambled_copy(scans[0])
    p.stage_scan(0, c0)
    _scramble(c0)  # the caller's arrays are free once staging returns
    for k in range(len(scans)):
        p.run_scan(k % 2, scans[k], k)
        if k + 1 < len(scans):  # the next scan's copy overlaps this scan's compute
            c = _scrambled_copy(scans[k + 1])
            p.stage_scan((k + 1) % 2, c)
            _scramble(c)
    ctx.sync()
    _assert_same(_state(p), want)


def test_restage_slot_of_a_queued_scan(ctx):
    """Slot 0 is restaged while the scan that reads it is still queued (and, second time, while
    its exchange is pending): the copy must wait for that scan's reads."""
    case = cases.build(H=16, n_az=1024, n_scans=3, io="computed")
    ref = _pipeline(case, ctx, 16, case["n"], True)
    for k, s in enumerate(case["scans"]):
        ref.stage_scan(0, s)
        ref.run_scan(0, s, k)
    ctx.sync()
    want = _state(ref)
    p = _pipeline(case, ctx, 16, case["n"], True)
    s0, s1, s2 = case["scans"]
    p.stage_scan(0, s0)
    p.run_scan(0, s0, 0)
    p.stage_scan(0, s1)             # scan 0 may still be running
    p.run_scan_local(0, s1, 1)
    p.stage_scan(0, s2)             # scan 1's exchange is pending
    p.finish_scan()
    p.run_scan(0, s2, 2)
    ctx.sync()
    _assert_same(_state(p), want)


def test_state_locked_between_scan_halves(ctx):
    case = cases.build(H=4, n_az=256, n_scans=2, io="computed")
    p = _pipeline(case, ctx, 4, case["n"], True)
    s0, s1 = case["scans"]
    p.stage_scan(0, s0)
    p.run_scan_local(0, s0, 0)
    iw = case["iw"]
    hy = case["hyp"]
    for call in (lambda: p.set_iw(*iw), lambda: p.set_weights(hy["weights"]), lambda: p.set_map(case["map_record"]),
                 lambda: p.set_beliefs(hy["X_anchor"], hy["z_lin"], hy["L"], hy["h"]), lambda: p.set_io_mode(True),
                 lambda: p.combined(), lambda: p.get_iw(), lambda: p.get_map(), lambda: p.run_scan_local(0, s0, 1)):
        with pytest.raises(ValueError, match="pending"):
            call()
    # allowed while pending: the partial record, per-hypothesis results, staging the next scan
    assert p.partial().shape[0] > 0
    p.get_beliefs()
    p.hyp_diag()
    p.stage_scan(1, s1)
    p.finish_scan()
    p.combined()
    p.run_scan(1, s1, 1)
    ctx.sync()
    with pytest.raises(ValueError, match="no timed exchange"):
        p.exchange_ms()
