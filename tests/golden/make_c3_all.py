#!/usr/bin/env python3
"""Generate tests/golden/c3_all.npz (TEST INFRASTRUCTURE): the oracle's first C3 scan for EVERY one of
the 256 hypotheses, so the -m gpu suite can compare all of them with the HIP pipeline without running
the oracle 256 times on the GPU box (tests/test_gpu_configs.py samples 4 per scan; VERDICT r4
"C3/C5 compare only 3-5 sampled hypotheses").

The case is oracle/cases.build(H=256, n_az=4096, n_scans=1, io="computed") — exactly the C3 bench
workload of test_c3_bench_workload_matches_oracle — and the oracle's inputs are the case's initial
state (beliefs, IW, map), which is what the pipeline holds before its first scan. The reference cannot
run here (no JAX): these are oracle outputs, not reference outputs.

Run from the repo root:  python tests/golden/make_c3_all.py   (8 worker processes, ~1 min)
"""

from __future__ import annotations

import hashlib
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))

from oracle import cases  # noqa: E402
from oracle import gc_oracle as O  # noqa: E402

H, N_AZ = 256, 4096
EPS_LIFT = 1e-9
_CASE = None


def _setup():
    global _CASE
    case = cases.build(H=H, n_az=N_AZ, n_scans=1, io="computed")
    nuP, PsiP, nuM, PsiM = case["iw"]
    mapst = O.MapStats(*(x.copy() for x in (case["state"].map.S_dir, case["state"].map.S_dir_scatter,
                                             case["state"].map.N_dir, case["state"].map.N_pos,
                                             case["state"].map.sum_p, case["state"].map.sum_ppT)))
    _CASE = dict(case=case, Q=O.iw_process_Q(nuP, PsiP), Sga=(O.iw_meas_mode(nuM, PsiM, 0), O.iw_meas_mode(nuM, PsiM, 1)),
                 mapst=mapst, md=O.map_derived(mapst), scan=cases.scan_input(case["scans"][0]),
                 cfg=O.PipeConfig(n_points_cap=case["n"]))
    return _CASE


def _one(i):
    c = _CASE
    hy = c["case"]["hyp"]
    b0 = O.Belief(hy["X_anchor"][i].copy(), hy["z_lin"][i].copy(), hy["L"][i].copy(), hy["h"][i].copy(),
                  float(hy["stamp"][i]))
    r = O.scan_hypothesis(b0, c["scan"], c["Q"], None, c["mapst"], c["md"], c["case"]["bins"], c["cfg"], c["Sga"])
    b = r["belief"]
    S = np.linalg.inv(b.L + EPS_LIFT * np.eye(b.L.shape[0]))
    return (np.asarray(r["pose"], np.float64), b.X_anchor.copy(), b.z_lin.copy(), S[0:6, 0:6].copy(),
            np.array([r["alpha"], r["beta"], r["T"], r["cond6"]]), np.asarray(r["xi_body"], np.float64))


def main():
    c = _setup()
    with Pool(min(8, os.cpu_count() or 1), initializer=_setup) as pool:
        out = pool.map(_one, range(H))
    pose, X, z, Sp, sc, xi = (np.stack([o[k] for o in out]) for k in range(6))
    s0 = c["case"]["scans"][0]
    h = hashlib.sha256()
    for a in (s0["points"], s0["timestamps"], s0["weights"], c["case"]["hyp"]["L"], c["case"]["hyp"]["X_anchor"],
              c["case"]["map_record"]):
        h.update(np.ascontiguousarray(a, np.float64).tobytes())
    np.savez_compressed(os.path.join(HERE, "c3_all.npz"), pose=pose, X_anchor=X, z_lin=z, Sigma_pose=Sp,
                        scalars=sc, xi_body=xi, input_sha256=np.frombuffer(h.digest(), np.uint8))
    print("wrote", os.path.join(HERE, "c3_all.npz"), pose.shape)


if __name__ == "__main__":
    main()
