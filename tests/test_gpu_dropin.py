"""The reference node's per-hypothesis operator chain through the device-resident per-operator
drop-ins (gcslam.dropin_node: backend_node.py:2036-2119 with the legacy bin wiring), against the
oracle's per-hypothesis scan (oracle/gc_oracle.py scan_hypothesis / process_scan) at the north-star bars,
and the arena: once warm, a scan of the chain performs no hipMalloc / hipFree (include/gcslam.h
gc_buffer_alloc; VERDICT r4 "device-resident per-operator drop-in path")."""

import numpy as np
import pytest

from oracle import cases
from oracle import gc_oracle as O

pytestmark = pytest.mark.gpu


def _node(case, ctx):
    from gcslam.belief import BeliefGaussianInfo
    from gcslam.constants import GC_CHART_ID
    from gcslam.dropin_node import BinMap, DropinNode, IOGiven
    from gcslam.ops import MeasurementNoiseIWState, ProcessNoiseIWState
    st = case["state"]
    hy = case["hyp"]
    beliefs = [BeliefGaussianInfo(GC_CHART_ID, "initial", hy["X_anchor"][i], hy["stamp"][i], hy["z_lin"][i], hy["L"][i],
                                  hy["h"][i]) for i in range(len(st.beliefs))]
    Lio, hio, cert = case["io"]
    ios = [IOGiven(Lio[i], hio[i], cert[i]) for i in range(len(beliefs))]
    node = DropinNode(beliefs, st.weights, case["bins"], _binmap(st.map), O.iw_process_Q(st.nu_proc, st.Psi_proc),
                      ProcessNoiseIWState(st.nu_proc.copy(), st.Psi_proc.copy()),
                      MeasurementNoiseIWState(st.nu_meas.copy(), st.Psi_meas.copy()), case["n"], ctx=ctx)
    return node, ios


def _binmap(m):
    from gcslam.dropin_node import BinMap
    mu_dir, kap, cen, Sc = O.map_derived(m)
    B = cen.shape[0]
    der = np.concatenate([mu_dir, np.asarray(kap).reshape(B, 1), cen, Sc.reshape(B, 9), np.zeros((B, 1))], axis=1)
    return BinMap(record=cases.map_to_record(m), derived=der)


def test_dropin_chain_matches_oracle(ctx):
    """K = 4 hypotheses, budget stride 2 (cap = half the scan), two scans with the IW feedback (the bin map
    is the oracle's between scans): per-hypothesis world pose within 1e-6 abs (the north-star bar), L
    within 1e-8 relative, the trigger sum T within 1e-7 relative and ξ_body within 1e-9."""
    case = cases.build(H=4, n_az=256, n_scans=2, cap=2048)
    node, ios = _node(case, ctx)
    st = case["state"]
    for k, s in enumerate(case["scans"]):
        res = node.process_scan(s, ios)
        st, comb, ref = O.process_scan(st, cases.scan_input(s), case["ios"], case["bins"], case["cfg"])
        for i, (r, o) in enumerate(zip(res, ref)):
            b = r["belief"]
            pose = b.world_pose(ctx=ctx)
            assert np.max(np.abs(pose - o["pose"])) <= 1e-6, (k, i, pose, o["pose"])
            assert np.max(np.abs(b.L - o["belief"].L)) <= 1e-8 * np.max(np.abs(o["belief"].L)), (k, i)
            assert abs(r["T"] - o["T"]) <= 1e-7 * abs(o["T"]) + 1e-12, (k, i, r["T"], o["T"])
            assert np.max(np.abs(r["xi"] - o["xi_body"])) <= 1e-9, (k, i)
        assert np.max(np.abs(node.combined.belief_out.L - comb["L"])) <= 1e-8 * np.max(np.abs(comb["L"]))
        assert np.max(np.abs(node.pn.Psi - st.Psi_proc)) <= 1e-7 * np.max(np.abs(st.Psi_proc)) + 1e-18
        # the measurement-IW state from the gyro / accel window statistics of every hypothesis
        assert np.max(np.abs(node.mn.Psi - st.Psi_meas)) <= 1e-9 * np.max(np.abs(st.Psi_meas)), k
        assert np.max(np.abs(node.mn.nu - st.nu_meas)) <= 1e-12 * np.max(np.abs(st.nu_meas)), k
        node.map = _binmap(st.map)


def test_dropin_chain_steady_state_allocates_nothing(ctx):
    """After one warm scan every device buffer of the chain comes from the context's arena: the next
    scans call hipMalloc / hipFree zero times (gc_ctx_alloc_stats), and the arena's live buffers return
    to their count before the scan."""
    import gc as _gc
    case = cases.build(H=4, n_az=256, n_scans=3, cap=2048)
    node, ios = _node(case, ctx)
    node.process_scan(case["scans"][0], ios)
    _gc.collect()
    a0 = ctx.alloc_stats()
    for s in case["scans"][1:]:
        node.process_scan(s, ios)
    _gc.collect()
    a1 = ctx.alloc_stats()
    assert a1["hip_mallocs"] == a0["hip_mallocs"], (a0, a1)
    assert a1["hip_frees"] == a0["hip_frees"], (a0, a1)
    assert a1["reuses"] > a0["reuses"]
    assert a1["live"] == a0["live"], (a0, a1)
