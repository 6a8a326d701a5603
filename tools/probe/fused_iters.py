"""Dev probe: the grid-form fused bins kernel (gc_scan_bins_fused) at C3 for explicit iteration
counts: per-task overhead = d(time) / d(tasks). Usage (GPU box): python3 tools/probe/fused_iters.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from gcslam import _abi  # noqa: E402
from gcslam.constants import GC_B_BINS, GC_TAU_SOFT_ASSIGN, T_BASE_LIDAR  # noqa: E402
from gcslam.ops.binning import create_fibonacci_atlas  # noqa: E402
from gcslam.synth import make_scan  # noqa: E402

ctx = _abi.Context(0)
H, B = int(sys.argv[1]) if len(sys.argv) > 1 else 256, GC_B_BINS
s = make_scan(1)
n = s["points"].shape[0]
rng = np.random.default_rng(5)
xi = np.zeros((H, 6)); xi[:, 0] = 0.1 + rng.normal(0, 0.005, H); xi[:, 5] = 0.03 + rng.normal(0, 0.002, H)
d = {k: _abi.DeviceArray.from_host(ctx, s[k]) for k in ("points", "timestamps", "weights")}
scal = _abi.DeviceArray(ctx, 8)
_abi.call("gc_budget_stats", ctx.handle, d["weights"].ptr, n, n, scal.ptr, ctx=ctx)
dx, db = _abi.DeviceArray.from_host(ctx, xi), _abi.DeviceArray.from_host(ctx, create_fibonacci_atlas(B).dirs)
st, ce = _abi.DeviceArray(ctx, (H, B, 38)), _abi.DeviceArray(ctx, (H, 8))
oa, op = _abi.f64p(np.asarray(T_BASE_LIDAR[:3]))
for iters in (16, 8, 4, 2, 1, 16):
    def launch():
        _abi.call("gc_scan_bins_fused", ctx.handle, H, n, n, B, d["points"].ptr, d["timestamps"].ptr,
                  d["weights"].ptr, scal.ptr, s["scan_start"], s["scan_end"], dx.ptr, db.ptr, GC_TAU_SOFT_ASSIGN, op,
                  1e-12, 1e-12, st.ptr, ce.ptr, iters, ctx=ctx)
    for _ in range(10):
        launch()
    ev = [_abi.Event(ctx) for _ in range(2)]
    ev[0].record()
    for _ in range(10):
        launch()
    ev[1].record()
    ctx.sync()
    ms = ev[0].elapsed_ms(ev[1]) / 10
    tasks = H * ((n + iters * 256 - 1) // (iters * 256))
    print(f"iters {iters:2d}  tasks {tasks:6d}  {ms:.4f} ms  ({ms * 1e3 / tasks * 512:.2f} us per task-slot)", flush=True)
