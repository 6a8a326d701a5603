"""Dev probe (GPU box): cost of the fused bins kernel's deskew forms. Times gc_scan_bins_fused
(65,536 points x 256 hypotheses, 48 bins, the benchmark geometry) with the scan twists of the bench
(|ω| ~ 0.03: the short series everywhere) against fast rotations (the nine-term series and the
sin / cos closed form in most waves). Usage: python3 tools/probe/deskew_rot_cost.py [lib]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))
sys.path.insert(0, ROOT)
from gcslam import _abi  # noqa: E402

if len(sys.argv) > 1:
    _abi.LIB_PATH = os.path.abspath(sys.argv[1])
from gcslam.synth import make_scan  # noqa: E402
from oracle import gc_oracle as O  # noqa: E402

ctx = _abi.Context(0)
s = make_scan(1, n_az=4096)
n = s["points"].shape[0]
H, B = 256, 48
bins = O.fibonacci_atlas(B)
dP, dT, dW = (_abi.DeviceArray.from_host(ctx, s[k]) for k in ("points", "timestamps", "weights"))
scal = _abi.DeviceArray(ctx, 8)
_abi.call("gc_budget_stats", ctx.handle, dW.ptr, n, n, scal.ptr, ctx=ctx)
dB = _abi.DeviceArray.from_host(ctx, bins)
st = _abi.DeviceArray(ctx, (H, B, 38))
ce = _abi.DeviceArray(ctx, (H, 8))
oa, op = _abi.f64p([-0.065447, -0.100474, 0.108987])
rng = np.random.default_rng(9)
cases = {"bench (|w| ~ 0.03)": rng.normal(size=(H, 6)) * 0.02,
         "series (|w| ~ 0.6)": np.hstack([rng.normal(size=(H, 3)) * 0.2, rng.normal(size=(H, 3)) * 0.35]),
         "closed form (|w| ~ 2.5)": np.hstack([rng.normal(size=(H, 3)) * 0.2, rng.normal(size=(H, 3)) * 1.5])}
ev = [_abi.Event(ctx) for _ in range(2)]
for name, xis in cases.items():
    dX = _abi.DeviceArray.from_host(ctx, xis)

    def run():
        _abi.call("gc_scan_bins_fused", ctx.handle, H, n, n, B, dP.ptr, dT.ptr, dW.ptr, scal.ptr,
                  s["scan_start"], s["scan_end"], dX.ptr, dB.ptr, 0.1, op, 1e-12, 1e-12, st.ptr, ce.ptr, 0, ctx=ctx)
    for _ in range(20):
        run()
    ctx.sync()
    reps = 30
    ev[0].record()
    for _ in range(reps):
        run()
    ev[1].record()
    ctx.sync()
    print(f"{name:26s} {ev[0].elapsed_ms(ev[1]) / reps:.4f} ms per call", flush=True)
