#!/bin/bash
# GPU box (round 4 dev): kernel trace of build_var/<v> at H hypotheses, per-scan timeline.
# Usage: bash tools/dev/r4_trace_var.sh <variant> [H]   Output: gpurun_out/r4/trace_<v>_h<H>/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
v=$1; H=${2:-32}
o=gpurun_out/r4/trace_${v}_h$H; rm -rf $o; mkdir -p $o
timeout -k 10 200 rocprofv3 --kernel-trace -d $o/kt -o kt --output-format csv -- python3 tools/dev/ab_bench.py fl-slam_amd/build_var/$v/libgcslam.so --hyps $H --no-cpu --no-roofline --no-map --no-c5 --no-extras --steps 50 --warmup 20 > $o/b.json 2> $o/b.err || exit 1
python3 tools/timeline.py "$(find $o/kt -name '*kernel_trace.csv' | head -1)" 14 > $o/timeline.txt
cat $o/timeline.txt
