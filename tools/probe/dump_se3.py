"""Dump the device se3_log / so3_log / se3_exp at the Lie test's large-angle grid (debug helper)."""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "fl-slam_amd"))
from gcslam import _abi  # noqa: E402
from gcslam.ops import se3  # noqa: E402

TH = [0.0, 1e-9, 9.9e-8, 1.01e-7, 1e-4, 0.01, 0.5, 1.0, 2.0, 2.5, 3.0, math.pi - 0.02, math.pi - 0.01,
      math.pi - 1e-4, math.pi - 1e-6, math.pi - 5e-8, math.pi - 1e-12, math.pi]
a = np.random.default_rng(7).normal(size=(12, 3))
a[0], a[1], a[2], a[3] = [1, 0, 0], [0, 0, 1], [0, 0, -1], [1, 1, 0]
ax = a / np.linalg.norm(a, axis=1, keepdims=True)
w = np.array([t * x for t in TH for x in ax])
t = np.random.default_rng(11).normal(size=w.shape) * 3.0
T = np.concatenate([t, w], 1)
ctx = _abi.Context()
out = dict(T=T, log=se3.se3_log(T, ctx=ctx), exp=se3.se3_exp(T, ctx=ctx), Vi=se3._se3_V_inv(w, ctx=ctx),
           R=se3.so3_exp(w, ctx=ctx))
out["so3log"] = se3.so3_log(out["R"], ctx=ctx)
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/dump_se3.npz", **out)
print("ok")
