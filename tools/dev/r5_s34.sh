#!/bin/bash
# GPU box (round 5 dev): per-phase / per-wave cycles of the chain kernels at H = 32 (build_var/timing, GC_PHASE_TIMING)
# after the DPP preintegration scans and the bins tier change, then tools/probe/lift_lat (the lift iteration's latency).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s34; rm -rf $o; mkdir -p $o
timeout -k 10 120 python3 tools/phase_timing.py 32 > $o/phases.txt 2>&1 || { tail -5 $o/phases.txt; exit 1; }
cat $o/phases.txt
timeout -k 10 60 tools/probe/lift_lat > $o/lift_lat.txt 2>&1 || { tail -5 $o/lift_lat.txt; exit 1; }
cat $o/lift_lat.txt
