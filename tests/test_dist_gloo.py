"""Multi-rank exchange logic on CPU (world_size 2, gloo): hypotheses sharded contiguously, each
rank packs its partial record in the device layout (gcslam.pipeline.RECORD), records are
all-gathered and reduced in rank order — the result must equal the unsharded combine.
The per-hypothesis math runs in the oracle here (no GPU); the GPU path shares the layout and
the reduction order (csrc/gc_evidence.hip k_combine_local / k_combine_final)."""

import os
import sys

import numpy as np
import pytest
import torch.distributed as td
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pack(case, res, h0, h1):
    from gcslam.pipeline import RECORD, partial_len
    from oracle import gc_oracle as O
    st = case["state"]
    H = len(st.beliefs)
    B = 48
    floor = 0.01 / H
    w = st.weights
    wsum = np.sum(np.maximum(w, floor))
    rec = np.zeros(partial_len(B))
    for k in range(h0, h1):
        r = res[k - h0]
        b = r["belief"]
        wn = max(w[k], floor) / wsum
        mu = O.chol_solve_lifted(b.L, b.h)[0]
        rec[slice(*RECORD["L"])] += wn * b.L.reshape(-1)
        rec[slice(*RECORD["h"])] += wn * b.h
        rec[slice(*RECORD["z"])] += wn * b.z_lin
        rec[slice(*RECORD["mu"])] += wn * mu
        rec[slice(*RECORD["mu2"])] += wn * float(mu @ mu)
        rec[slice(*RECORD["dPsiP"])] += w[k] * r["dPsiP"].reshape(-1) if "dPsiP" in r else w[k] * r["dPsi_proc"].reshape(-1)
        rec[slice(*RECORD["dnuP"])] += w[k] * r["dnu_proc"]
        rec[slice(*RECORD["dPsiM"])] += w[k] * r["dPsi_meas"].reshape(-1)
        rec[slice(*RECORD["dnuM"])] += w[k] * r["dnu_meas"]
    if h0 == 0:
        rec[slice(*RECORD["X0"])] = res[0]["belief"].X_anchor
        from oracle import cases
        rec[848:848 + 26 * B] = cases.map_to_record(res[0]["map_inc"]).reshape(-1)
    return rec


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))
    sys.path.insert(0, ROOT)
    import torch
    from gcslam.pipeline import shard, RECORD
    from oracle import cases, gc_oracle as O
    td.init_process_group("gloo", rank=rank, world_size=world)
    case = cases.build(H=6, n_az=128, n_scans=1)
    st, s = case["state"], case["scans"][0]
    H = len(st.beliefs)
    h0, h1 = shard(H, rank, world)
    Q = O.iw_process_Q(st.nu_proc, st.Psi_proc)
    md = O.map_derived(st.map)
    res = [O.scan_hypothesis(st.beliefs[k], cases.scan_input(s), Q, case["ios"][k], st.map, md, case["bins"],
                             case["cfg"]) for k in range(h0, h1)]
    rec = torch.from_numpy(_pack(case, res, h0, h1))
    gathered = [torch.zeros_like(rec) for _ in range(world)]
    td.all_gather(gathered, rec)
    red = np.zeros_like(rec.numpy())
    for g in range(world):  # rank order, as k_combine_final
        red = red + gathered[g].numpy()
    L, _ = O.psd_project(red[slice(*RECORD["L"])].reshape(22, 22))
    q.put((rank, h0, h1, L, red))
    td.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_exchange_equals_unsharded_combine(world):
    sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))
    from gcslam.pipeline import RECORD, shard
    from oracle import cases, gc_oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + world
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    case = cases.build(H=6, n_az=128, n_scans=1)
    st2, comb, res = O.process_scan(case["state"], cases.scan_input(case["scans"][0]), case["ios"],
                                    case["bins"], case["cfg"])
    ranges = sorted((o[1], o[2]) for o in outs)
    assert ranges == [shard(6, r, world) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == 6 and all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    Ls = [o[3] for o in outs]
    for L in Ls[1:]:
        assert np.array_equal(L, Ls[0])  # bit-identical on every rank
    # summation order differs from the unsharded einsum: rounding-level agreement
    np.testing.assert_allclose(Ls[0], comb["L"], rtol=0, atol=1e-12 * np.max(np.abs(comb["L"])))
    red = outs[0][4]
    np.testing.assert_allclose(red[slice(*RECORD["h"])], comb["h"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(red[slice(*RECORD["z"])], comb["z_lin"], rtol=1e-12, atol=1e-14)
    # IW statistics: Σ_h w_h dΨ equals the unsharded accumulation
    aP = sum(case["state"].weights[i] * res[i]["dPsi_proc"] for i in range(6))
    np.testing.assert_allclose(red[slice(*RECORD["dPsiP"])].reshape(7, 6, 6), aP, rtol=1e-12, atol=1e-30)
    # map increments come from hypothesis 0's owner only
    np.testing.assert_allclose(red[848:848 + 26 * 48].reshape(48, 26), cases.map_to_record(res[0]["map_inc"]),
                               rtol=0, atol=0)
