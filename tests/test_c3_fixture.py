"""tests/golden/c3_all.npz and c5_all.npz (the oracle's first C3 / C5 scan for every hypothesis, read
by test_c{3,5}_every_hypothesis_matches_fixture on the GPU) are pinned here on the CPU: their inputs
hash to the current oracle/cases.build case, and the current oracle reproduces two hypotheses of each
to 1e-12 (BLAS thread counts may reorder a few sums; a later oracle or case edit that changes them
fails here, not as a GPU mismatch)."""

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


@pytest.mark.parametrize("name,hyps", [("c3", (0, 200)), ("c5", (0, 1023))])
def test_fixture_is_the_current_case_and_oracle(name, hyps):
    import make_c3_all as M
    g = np.load(os.path.join(ROOT, "tests", "golden", f"{name}_all.npz"))
    c = M._setup(name)
    assert bytes(g["input_sha256"]) == M.input_digest(c)
    H = M.CONFIGS[name]["H"]
    assert g["pose"].shape == (H, 6) and np.all(np.isfinite(g["Sigma_pose"]))
    for i in hyps:
        pose, X, z, Sp, sc, xi = M._one(i)
        for a, b in ((pose, g["pose"][i]), (X, g["X_anchor"][i]), (z, g["z_lin"][i]), (Sp, g["Sigma_pose"][i]),
                     (sc, g["scalars"][i]), (xi, g["xi_body"][i])):
            np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-15)
