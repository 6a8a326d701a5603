"""Dev helper: phase cycle counts of the IMU/odom branch workgroups (io_branch_wg inside k_bins_io)
from a library built with -DGC_IO_TIMING (tools/probe/libgcslam_iot.so):
    make -C fl-slam_amd BUILD=build_iot OUT=../tools/probe/libgcslam_iot.so \\
        CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include -DGC_IO_TIMING"
Runs the bench workload (64k points x H hypotheses, branch computed); prints per-phase cycles of
hypothesis 0 and the spread of the branch's total over all hypotheses."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))
sys.path.insert(0, ROOT)
from gcslam import _abi  # noqa: E402

_abi.LIB_PATH = os.path.join(ROOT, "tools", "probe", "libgcslam_iot.so")
import numpy as np  # noqa: E402
import bench  # noqa: E402

from gcslam.constants import GC_B_BINS, T_BASE_LIDAR  # noqa: E402
from gcslam.ops.binning import create_fibonacci_atlas  # noqa: E402
from gcslam.pipeline import BatchedScanPipeline, PipelineConfig, iw_meas_prior, iw_process_prior  # noqa: E402
from gcslam.synth import make_hypotheses, make_scan  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 32
ctx = _abi.Context(0)
B = GC_B_BINS
origin = np.asarray(T_BASE_LIDAR[:3])
scans = [make_scan(k + 1) for k in range(3)]
n = scans[0]["points"].shape[0]
pipe = BatchedScanPipeline(H, n, PipelineConfig(n_points_cap=n), ctx=ctx)
hy = make_hypotheses(H)
pipe.set_beliefs(hy["X_anchor"], hy["z_lin"], hy["L"], hy["h"], hy["stamp"])
pipe.set_weights(hy["weights"])
pipe.set_io_mode(True)
pipe.set_iw(*iw_process_prior(), *iw_meas_prior())
pipe.set_map(bench.warmup_map_record(ctx, _abi, make_scan(0), n, B, create_fibonacci_atlas(B).dirs, origin))
for k, s in enumerate(scans):
    pipe.stage_scan(k, s)
for r in range(6):
    pipe.run_scan(r % 3, scans[r % 3], r)
ctx.sync()
q = np.asarray(pipe.io_parts())[:, 30:35]
d = np.diff(q, axis=1)
names = ["window+preintegrate", "vMF gravity", "factors (per lane)", "sum+certs"]
for k, nm in enumerate(names):
    print(f"{nm:24s} hyp0 {d[0, k]:9.0f}  median {np.median(d[:, k]):9.0f}  max {d[:, k].max():9.0f} cycles")
tot = q[:, 4] - q[:, 0]
print(f"branch total: median {np.median(tot):.0f} max {tot.max():.0f} cycles; start spread {q[:, 0].max() - q[:, 0].min():.0f}")
