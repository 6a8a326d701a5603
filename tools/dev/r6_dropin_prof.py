"""Dev (GPU box, round 6): host profile of the per-operator drop-in leg (bench.py dropin_leg) — cProfile
of the timed scans, top functions by total time, plus the leg's own ms/scan. Writes to argv[1]."""

import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))

import bench  # noqa: E402
from gcslam import _abi  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/dropin_prof.txt"
ctx = _abi.Context(0)
r0 = bench.dropin_leg(ctx, _abi)
pr = cProfile.Profile()
pr.enable()
r = bench.dropin_leg(ctx, _abi, warm=1, scans=10)
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(45)
s2 = io.StringIO()
pstats.Stats(pr, stream=s2).sort_stats("cumulative").print_stats(60)
with open(out, "w") as f:
    f.write("plain: %.3f ms/scan; profiled: %.3f ms/scan\n" % (r0["ms_per_scan"], r["ms_per_scan"]))
    f.write(s.getvalue())
    f.write(s2.getvalue())
print("dropin ms/scan", r0["ms_per_scan"])
