#!/bin/bash
# Dev (GPU box): kernel timeline of one scan of the batched pipeline at H hypotheses (rocprofv3
# kernel trace of a short bench run). Usage: bash tools/trace_scan.sh <H> [tag]
set -e
H=${1:-32}; tag=${2:-h$H}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/trace_$tag; rm -rf $o; mkdir -p $o
timeout -k 10 200 rocprofv3 --kernel-trace -d $o/kt -o kt --output-format csv -- python3 bench.py --hyps $H --no-cpu --no-roofline --no-map --no-c5 --no-dropin --no-extras --steps 50 --warmup 20 > $o/bench.json 2> $o/bench.err
python3 tools/timeline.py "$(find $o/kt -name '*kernel_trace.csv' | head -1)" 8 > $o/timeline.txt
cat $o/timeline.txt
