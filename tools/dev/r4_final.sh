#!/bin/bash
# GPU box, round 4 final evidence in one call: the -m gpu suite, the default bench line, the same
# command under rocprofv3 --kernel-trace --stats, the H = 32 line, kernel traces + timelines at
# H = 256 / 32, PMC traffic of the contract pair and of the C5 map kernels. Every step has its own
# time limit; a fault, abort or time limit ends the script. Output: gpurun_out/r4/final/ (+ pmc_*).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4/final; rm -rf $o; mkdir -p $o
stop() { case $1 in 0) ;; *) echo "stopped rc=$1 at $2" | tee -a $o/summary.txt; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $o/gpu_tests.txt 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $o/gpu_tests.txt)" | tee -a $o/summary.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 420 python3 bench.py > $o/bench.json 2> $o/bench.err; stop $? bench
echo "bench $(tail -1 $o/bench.json | cut -c1-260)" | tee -a $o/summary.txt
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $o/kt_bench -o kt --output-format csv -- python3 bench.py --no-cpu > $o/bench_rocprof.json 2> $o/bench_rocprof.err; stop $? bench_rocprof
cp "$(find $o/kt_bench -name '*kernel_stats.csv' | head -1)" $o/kernel_stats_bench.csv; find $o/kt_bench -name "*kernel_trace.csv" -delete
timeout -k 10 180 python3 bench.py --hyps 32 --no-cpu --no-map --no-c5 --no-roofline --steps 400 --warmup 50 > $o/bench_h32.json 2>> $o/bench.err; stop $? bench_h32
for H in 256 32; do
  d=$o/kt_h$H
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o kt --output-format csv -- python3 bench.py --hyps $H --no-cpu --no-roofline --no-map --no-c5 --no-extras --steps 50 --warmup 20 > $d.json 2> $d.err; stop $? kt_h$H
  python3 tools/timeline.py "$(find $d -name '*kernel_trace.csv' | head -1)" 14 > $o/timeline_h$H.txt
  cp "$(find $d -name '*kernel_stats.csv' | head -1)" $o/kernel_stats_h$H.csv
  find $d -name "*kernel_trace.csv" -delete
done
bash tools/pmc_traffic.sh r04 > $o/pmc_traffic.log 2>&1; stop $? pmc_traffic
cp gpurun_out/pmc_traffic_r04.json $o/pmc_traffic.json
bash tools/pmc_fuse.sh r04 > $o/pmc_fuse.log 2>&1; stop $? pmc_fuse
cp gpurun_out/pmc_fuse_r04.json $o/pmc_fuse.json
rm -rf gpurun_out/pmc_traffic gpurun_out/pmc_fuse
cat $o/summary.txt
