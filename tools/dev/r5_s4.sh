#!/bin/bash
# GPU box (round 5 dev): per-phase cycles of the chain kernels (GC_PHASE_TIMING build) and the
# per-workgroup / per-task trace of the bins launch (GC_BINS_TIMING build) at H hypotheses.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
H=${1:-32}
o=gpurun_out/r5s4_h$H; rm -rf $o; mkdir -p $o
timeout -k 10 120 python3 tools/phase_timing.py $H > $o/phases.txt 2>&1 || { cat $o/phases.txt; exit 1; }
cat $o/phases.txt
timeout -k 10 120 python3 tools/probe/bins_trace.py fl-slam_amd/build_var/btime/libgcslam.so $H > $o/bins_trace.txt 2>&1 || { tail $o/bins_trace.txt; exit 1; }
head -12 $o/bins_trace.txt; tail -14 $o/bins_trace.txt
