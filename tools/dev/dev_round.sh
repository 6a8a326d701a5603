#!/bin/bash
# Dev (GPU box): the Lie-map probe, the full -m gpu suite, per-phase cycles at H = 32 and the
# H = 32 / H = 256 bench steps. Stops after a fault, abort or time limit.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/dev; rm -rf $o; mkdir -p $o
stop() { case $1 in 124|134|137|139) echo "stopped rc=$1" >> $o/summary.txt; exit $1;; esac; }
timeout -k 5 60 ./tools/probe/probe_lie > $o/probe_lie.txt 2>&1; stop $?
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.txt 2>&1; rc=$?; echo "tests rc=$rc $(tail -1 $o/gpu_tests.txt)" >> $o/summary.txt; stop $rc
timeout -k 10 150 python3 tools/phase_timing.py 32 > $o/phases_h32.txt 2>&1; stop $?
for H in 32 256; do
  timeout -k 10 180 python3 bench.py --hyps $H --no-cpu --no-map --no-c5 --no-roofline --steps 300 --warmup 50 > $o/bench_h$H.json 2>>$o/bench.err; stop $?
  echo "H=$H $(tail -1 $o/bench_h$H.json | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")" >> $o/summary.txt
done
