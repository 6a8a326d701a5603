#!/bin/bash
# Dev (GPU box): smoke(), the C2 (H = 1) and shard (H = 32) bench steps for BASELINE.md.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/extra; rm -rf $o; mkdir -p $o
stop() { case $1 in 124|134|137|139) echo "stopped rc=$1" >> $o/summary.txt; exit $1;; esac; }
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1; rc=$?; echo "smoke rc=$rc $(tail -1 $o/smoke.txt)" >> $o/summary.txt; stop $rc
for H in 1 32; do
  timeout -k 10 180 python3 bench.py --hyps $H --no-cpu --no-map --no-c5 --no-roofline --steps 400 --warmup 50 > $o/bench_h$H.json 2>>$o/bench.err; stop $?
  echo "H=$H $(tail -1 $o/bench_h$H.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])")" >> $o/summary.txt
done
cat $o/summary.txt
