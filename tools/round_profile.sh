#!/bin/bash
# Round evidence on the GPU box: gpu tests, default bench line, rocprofv3 kernel-trace stats of the
# same bench command, PMC traffic of the contract pair. Usage (GPU box): bash tools/round_profile.sh r01
# Outputs under gpurun_out/<round>/ (then copied into profiles/<round>/ by hand).
set -e
round=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$round
rm -rf $out; mkdir -p $out
# a failing assertion does not stop the evidence run; a fault, abort or time limit does
rc=0; timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || rc=$?
tail -2 $out/gpu_tests.log
case $rc in 124|134|137|139) echo "gpu tests stopped rc=$rc"; exit $rc;; esac
timeout -k 10 300 python3 bench.py > $out/bench.json 2> $out/bench.err
tail -c 400 $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- python3 bench.py --no-cpu > $out/bench_rocprof.json 2> $out/bench_rocprof.err
cp "$(find $out/kt -name '*kernel_stats.csv' | head -1)" $out/kernel_stats.csv
bash tools/pmc_traffic.sh $round
cp gpurun_out/pmc_traffic_$round.json $out/pmc_traffic.json
bash tools/pmc_fuse.sh $round
cp gpurun_out/pmc_fuse_$round.json $out/pmc_fuse.json
bash tools/trace_scan.sh 32 h32 > /dev/null && cp gpurun_out/trace_h32/timeline.txt $out/timeline_h32.txt
bash tools/trace_scan.sh 256 h256 > /dev/null && cp gpurun_out/trace_h256/timeline.txt $out/timeline_h256.txt
