#!/bin/bash
# Dev (GPU box): kernel + memory-copy timeline of the batched pipeline with per-step ingest and
# without, at H hypotheses. Usage: bash tools/dev/ingest_trace.sh <H> [tag]
set -e
H=${1:-32}; tag=${2:-h$H}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/ingest_$tag; rm -rf $o; mkdir -p $o
for mode in ingest noingest; do
  flag=""; [ $mode = noingest ] && flag="--no-ingest"
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $o/$mode -o kt --output-format csv -- python3 bench.py --hyps $H --no-cpu --no-roofline --no-map --no-c5 --steps 50 --warmup 20 $flag > $o/$mode.json 2> $o/$mode.err
  python3 tools/timeline.py "$(find $o/$mode -name '*kernel_trace.csv' | head -1)" 14 > $o/timeline_$mode.txt
done
tail -n 14 $o/timeline_*.txt; find $o -name '*memory_copy_trace.csv' | head -2
