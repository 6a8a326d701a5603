#!/usr/bin/env python3
"""Generate tests/golden/c3_all.npz and c5_all.npz (TEST INFRASTRUCTURE): the oracle's first scan for
EVERY hypothesis of C3 (256) and C5 (1024), so the -m gpu suite can compare all of them with the HIP
pipeline without running the oracle per hypothesis on the GPU box (tests/test_gpu_configs.py samples
3-5 per scan; VERDICT r4 "C3/C5 compare only 3-5 sampled hypotheses").

The cases are oracle/cases.build(H=256, n_az=4096, n_scans=1, io="computed") — the C3 bench workload of
test_c3_bench_workload_matches_oracle — and cases.build(H=1024, n_az=8192, n_scans=1, io="computed",
cap=65536) — test_c5_shape_matches_oracle's; the oracle's inputs are the case's initial state
(beliefs, IW, map), which is what the pipeline holds before its first scan. The reference cannot run
here (no JAX): these are oracle outputs, not reference outputs.

Run from the repo root:  python tests/golden/make_c3_all.py [c3|c5|all]   (8 worker processes; C3 ~1
min, C5 ~3 min)
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

CONFIGS = {"c3": dict(H=256, n_az=4096, cap=None), "c5": dict(H=1024, n_az=8192, cap=65536)}
EPS_LIFT = 1e-9
_CASE = None


def _setup(name="c3"):
    global _CASE
    cf = CONFIGS[name]
    case = cases.build(H=cf["H"], n_az=cf["n_az"], n_scans=1, io="computed", cap=cf["cap"])
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


def input_digest(c):
    s0 = c["case"]["scans"][0]
    h = hashlib.sha256()
    for a in (s0["points"], s0["timestamps"], s0["weights"], c["case"]["hyp"]["L"], c["case"]["hyp"]["X_anchor"],
              c["case"]["map_record"]):
        h.update(np.ascontiguousarray(a, np.float64).tobytes())
    return h.digest()


def make(name):
    c = _setup(name)
    H = CONFIGS[name]["H"]
    with Pool(min(8, os.cpu_count() or 1), initializer=_setup, initargs=(name,)) as pool:
        out = pool.map(_one, range(H))
    pose, X, z, Sp, sc, xi = (np.stack([o[k] for o in out]) for k in range(6))
    f = os.path.join(HERE, f"{name}_all.npz")
    np.savez_compressed(f, pose=pose, X_anchor=X, z_lin=z, Sigma_pose=Sp, scalars=sc, xi_body=xi,
                        input_sha256=np.frombuffer(input_digest(c), np.uint8))
    print("wrote", f, pose.shape)


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    for nm in (CONFIGS if which == "all" else [which]):
        make(nm)
