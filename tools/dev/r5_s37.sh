#!/bin/bash
# GPU box (round 5 dev): per-workgroup and per-task timing of the bins launch at H = 32 and 256 with the round's final
# tiers (build_var/btime, GC_BINS_TIMING).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s37; rm -rf $o; mkdir -p $o
for H in 32 256; do
  timeout -k 10 120 python3 tools/probe/bins_trace.py fl-slam_amd/build_var/btime/libgcslam.so $H > $o/bins_trace_h$H.txt 2>&1 || { tail $o/bins_trace_h$H.txt; exit 1; }
  sed -n 2,12p $o/bins_trace_h$H.txt; tail -14 $o/bins_trace_h$H.txt
done
