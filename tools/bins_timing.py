"""Dev helper: per-workgroup timing of the persistent bins launch (k_bins_io) from a library built
with -DGC_BINS_TIMING (tools/probe/libgcslam_bt.so):
    make -C fl-slam_amd BUILD=build_bt OUT=../tools/probe/libgcslam_bt.so \\
        CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include -DGC_BINS_TIMING"
Runs the bench workload (64k points x H hypotheses, IMU/odom branch computed) and prints, in cycles
from the first workgroup's start: the dispatch spread, prologue, finishing spread of the pullers,
tasks and iterations per puller, and the branch workgroups' end."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))
sys.path.insert(0, ROOT)
from gcslam import _abi  # noqa: E402

_abi.LIB_PATH = os.path.join(ROOT, "tools", "probe", "libgcslam_bt.so")
import numpy as np  # noqa: E402
import bench  # noqa: E402
from gcslam.constants import GC_B_BINS, T_BASE_LIDAR  # noqa: E402
from gcslam.ops.binning import create_fibonacci_atlas  # noqa: E402
from gcslam.pipeline import BatchedScanPipeline, PipelineConfig, iw_meas_prior, iw_process_prior  # noqa: E402
from gcslam.synth import make_hypotheses, make_scan  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 32
ctx = _abi.Context(0)
B = GC_B_BINS
scans = [make_scan(k + 1) for k in range(3)]
n = scans[0]["points"].shape[0]
pipe = BatchedScanPipeline(H, n, PipelineConfig(n_points_cap=n), ctx=ctx)
hy = make_hypotheses(H)
pipe.set_beliefs(hy["X_anchor"], hy["z_lin"], hy["L"], hy["h"], hy["stamp"])
pipe.set_weights(hy["weights"])
pipe.set_io_mode(True)
pipe.set_iw(*iw_process_prior(), *iw_meas_prior())
pipe.set_map(bench.warmup_map_record(ctx, _abi, make_scan(0), n, B, create_fibonacci_atlas(B).dirs,
                                     np.asarray(T_BASE_LIDAR[:3])))
for k, s in enumerate(scans):
    pipe.stage_scan(k, s)
for r in range(6):
    pipe.run_scan(r % 3, scans[r % 3], r)
ctx.sync()
nwg = H + 2 * 256
buf = np.zeros(8192 * 5)
L = _abi.lib()
L.gc_debug_bins_timing.argtypes = [C.c_void_p, C.c_int64]
assert L.gc_debug_bins_timing(buf.ctypes.data, buf.size) == 0
d = buf.reshape(8192, 5)[:nwg]
t0 = d[:, 0].min()
io, pl = d[d[:, 3] < 0], d[d[:, 3] >= 0]
q = lambda x: "min %8.0f  med %8.0f  max %8.0f" % (np.min(x), np.median(x), np.max(x))
print(f"H={H}: {len(io)} branch workgroups, {len(pl)} pullers")
print("branch start     ", q(io[:, 0] - t0))
print("branch end       ", q(io[:, 2] - t0))
print("puller start     ", q(pl[:, 0] - t0))
print("puller prologue  ", q(pl[:, 1] - pl[:, 0]))
print("puller end       ", q(pl[:, 2] - t0))
print("puller busy      ", q(pl[:, 2] - pl[:, 1]))
print("tasks/puller     ", q(pl[:, 3]))
print("iters/puller     ", q(pl[:, 4]))
busy = pl[:, 2] - pl[:, 1]
print("cycles/iteration  median %.0f" % np.median(busy / np.maximum(pl[:, 4], 1)))
