#!/bin/bash
# GPU box, round 4 evidence: the default bench line, the H = 32 shard line, kernel-trace stats and
# per-scan timelines at H = 256 and H = 32. Every step has its own time limit; a fault, abort or
# time limit ends the script. Output: gpurun_out/r4/ev/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4/ev; rm -rf $o; mkdir -p $o
stop() { case $1 in 0) ;; *) echo "stopped rc=$1 at $2" >> $o/summary.txt; exit $1;; esac; }
timeout -k 10 420 python3 bench.py > $o/bench.json 2> $o/bench.err; stop $? bench
echo "bench $(tail -1 $o/bench.json | cut -c1-300)" >> $o/summary.txt
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $o/kt_bench -o kt --output-format csv -- python3 bench.py --no-cpu > $o/bench_rocprof.json 2> $o/bench_rocprof.err; stop $? bench_rocprof
cp "$(find $o/kt_bench -name '*kernel_stats.csv' | head -1)" $o/kernel_stats_bench.csv; find $o/kt_bench -name "*kernel_trace.csv" -delete
timeout -k 10 180 python3 bench.py --hyps 32 --no-cpu --no-map --no-c5 --no-roofline --steps 400 --warmup 50 > $o/bench_h32.json 2>> $o/bench.err; stop $? bench_h32
for H in 256 32; do
  d=$o/kt_h$H
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o kt --output-format csv -- python3 bench.py --hyps $H --no-cpu --no-roofline --no-map --no-c5 --no-extras --steps 50 --warmup 20 > $d.json 2> $d.err; stop $? kt_h$H
  python3 tools/timeline.py "$(find $d -name '*kernel_trace.csv' | head -1)" 14 > $o/timeline_h$H.txt
  cp "$(find $d -name '*kernel_stats.csv' | head -1)" $o/kernel_stats_h$H.csv
done
cat $o/summary.txt
