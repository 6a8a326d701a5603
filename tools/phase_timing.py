"""Dev helper: per-phase cycle counts of hypothesis 0's workgroup in k_predict_imu (slots 0-8) and
k_evidence (10-19) and k_combine_final (20-25), from a library built with -DGC_PHASE_TIMING
(fl-slam_amd/build_var/timing/libgcslam.so, or $GC_TIMING_LIB):
    make -C fl-slam_amd BUILD=build_timing OUT=build_var/timing/libgcslam.so \
        CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include -DGC_PHASE_TIMING"
Runs the bench workload (64k points x 256 hypotheses) with the IMU/odom branch given (GC_IO_GIVEN
leaves io_parts to the instrumentation)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))
sys.path.insert(0, ROOT)
from gcslam import _abi  # noqa: E402

_abi.LIB_PATH = os.environ.get("GC_TIMING_LIB", os.path.join(ROOT, "fl-slam_amd", "build_var", "timing", "libgcslam.so"))
import numpy as np  # noqa: E402
from gcslam.pipeline import BatchedScanPipeline, PipelineConfig, iw_meas_prior, iw_process_prior  # noqa: E402
from gcslam.synth import make_hypotheses, make_io_evidence, make_scan  # noqa: E402
from oracle import cases  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ctx = _abi.Context(0)
scans = [make_scan(k + 1) for k in range(3)]
n = scans[0]["points"].shape[0]
pipe = BatchedScanPipeline(H, n, PipelineConfig(n_points_cap=n), ctx=ctx)
hy = make_hypotheses(H)
pipe.set_beliefs(hy["X_anchor"], hy["z_lin"], hy["L"], hy["h"], hy["stamp"])
# the given evidence without dt / extrinsic information, as the computed branch's (the excitation
# scales are then 0 and k_evidence takes the bench's path: μ_pred from predict, no extra factorization)
Lio, hio, cio = make_io_evidence(H)
Lio[:, 15:, :] = 0.0
Lio[:, :, 15:] = 0.0
hio[:, 15:] = 0.0
pipe.set_io_evidence(Lio, hio, cio)
pipe.set_iw(*iw_process_prior(), *iw_meas_prior())
m0 = cases.warmup_map(make_scan(0), n, np.asarray(pipe.cfg.lidar_origin), cases.O.fibonacci_atlas(48))
pipe.set_map(cases.map_to_record(m0))
for k, s in enumerate(scans):
    pipe.stage_scan(k, s)
for r in range(6):
    pipe.run_scan(r % 3, scans[r % 3], r)
ctx.sync()
t = pipe.io_parts().reshape(-1)  # hypothesis 0's slots, then hypothesis 1's (40+: preint marks)
names = {1: "predict: loads (Σ', μ, IMU)", 2: "predict: Σ' cert + lift solves + pose0", 3: "predict: (fallback chain)", 4: "predict: -",
         5: "predict: moments+dt_imu", 6: "predict: preintegrate", 7: "predict: xi+omega", 8: "predict: meas IW",
         11: "evidence: start..MF", 12: "evidence: MF..planar", 13: "evidence: L_raw,beta,excitation",
         14: "evidence: pose6 cond+alpha", 15: "evidence: fusion PSD", 16: "evidence: recompose+IW stats",
         17: "evidence: IW solves/inverse", 18: "evidence: map increment", 19: "evidence: drift+final solves",
         21: "combine wg0: reduce + 22x22 PSD", 23: "combine wg2: process IW apply",
         24: "combine wg2: meas IW apply", 25: "combine wg2: Q rebuild"}

for a, b, nm in ((10, 30, "evidence: MF rows"), (30, 31, "evidence: MF sum_bins"), (31, 11, "evidence: mf_finalize"),
                 (11, 32, "evidence: planar rows"), (32, 33, "evidence: planar sum_bins"),
                 (33, 12, "evidence: planar_finalize")):
    if t[a] and t[b]:
        print(f"{nm:36s} {t[b] - t[a]:10.0f} cycles")
for a, b, nm in ((5, 40, "predict: preint: 2 x so3_exp"), (40, 41, "predict: preint: rotation scan"),
                 (41, 42, "predict: preint: velocity scan"), (42, 43, "predict: preint: position terms"),
                 (43, 6, "predict: preint: sums")):
    if t[a] and t[b]:
        print(f"{nm:36s} {t[b] - t[a]:10.0f} cycles")
for a, b, nm in ((17, 34, "evidence: map inc: zt, R (lane 64)"), (34, 35, "evidence: map inc: pushforward"),
                 (17, 36, "evidence: drift: X_fin (lane 0)"), (36, 37, "evidence: drift: h_fin, μ_fin")):
    if t[a] and t[b]:
        print(f"{nm:36s} {t[b] - t[a]:10.0f} cycles")
# per-wave marks inside two phases (slots free on the split-predict route; 51-52 in hypothesis 1's area)
for a, b, nm in ((1, 26, "predict: Σ' chol cert (wave 0)"), (1, 27, "predict: lift μ_inc (wave 1)"),
                 (1, 28, "predict: lift σ_warp + dt_imu (wave 2)"), (1, 29, "predict: pose0, R0 (lane 192)"),
                 (14, 9, "evidence: fusion chol (wave 0)"), (9, 38, "evidence: δz solve (wave 0)"),
                 (9, 39, "evidence: Σ phase 1 + trace (wave 1)"), (15, 51, "evidence: recompose (lane 0)"),
                 (15, 52, "evidence: Σ phase 2 (waves 1-3)")):
    if t[a] and t[b]:
        print(f"{nm:36s} {t[b] - t[a]:10.0f} cycles")
for i in sorted(names):
    if t[i] and t[i - 1]:
        print(f"{names[i]:36s} {t[i] - t[i - 1]:10.0f} cycles")
# combine_final's workgroups 0 (slots 20-21) and 2 (22-25) run side by side: their counters are
# compared only within a workgroup
for a, b, nm in ((20, 49, "combine wg0: whole (record, barycenter, certs)"), (44, 45, "combine wg1: map update + derive"),
                 (48, 25, "combine wg2: whole (process IW, Q)"), (46, 47, "combine wg3: meas IW apply")):
    if t[a] and t[b]:
        print(f"{nm:36s} {t[b] - t[a]:10.0f} cycles")
print("predict total", t[8] - t[0], "evidence 10..19", t[19] - t[10], "combine wg0 20..21", t[21] - t[20],
      "combine wg2 22..25", t[25] - t[22])
