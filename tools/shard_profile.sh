#!/bin/bash
# Dev (GPU box): per-phase cycle counts (GC_PHASE_TIMING build) and the kernel timeline of one scan
# for a hypothesis shard. Usage: bash tools/shard_profile.sh <H> [tag]
set -e
H=${1:-32}; tag=${2:-h$H}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/shard_$tag; rm -rf $o; mkdir -p $o
timeout -k 10 120 python3 tools/phase_timing.py $H > $o/phases.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d $o/kt -o kt --output-format csv -- python3 bench.py --hyps $H --no-cpu --no-roofline --no-map --no-c5 --no-dropin --no-extras --steps 50 --warmup 20 > $o/bench.json 2> $o/bench.err
python3 tools/timeline.py "$(find $o/kt -name '*kernel_trace.csv' | head -1)" 9 > $o/timeline.txt
cat $o/phases.txt $o/timeline.txt; tail -c 300 $o/bench.json
