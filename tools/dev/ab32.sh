#!/bin/bash
# Dev (GPU box): per-phase cycles at H = 32 (timing build), then an interleaved A/B of the bins task
# geometry variants (build_var/*) at H = 32 and H = 256. Stops after a fault, abort or time limit.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/ab; rm -rf $o; mkdir -p $o
stop() { case $1 in 124|134|137|139) echo "stopped rc=$1" >> $o/ab.txt; exit $1;; esac; }
timeout -k 10 150 python3 tools/phase_timing.py 32 > $o/phases_h32.txt 2>&1; stop $?
run() {  # variant H tag extra-args
  if [ $1 = base ]; then L=fl-slam_amd/gcslam/libgcslam.so; else L=fl-slam_amd/build_var/$1/libgcslam.so; fi
  timeout -k 10 180 python3 tools/dev/ab_bench.py $L --hyps $2 --no-cpu --no-map --no-c5 ${@:4} > $o/$1_$3.json 2>>$o/ab.err; rc=$?; stop $rc
  echo "$1 H=$2 $(tail -1 $o/$1_$3.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print(d['ms_per_step'], (r.get('per_kernel') or {}).get('soft_assign', {}).get('GB/s'))")" >> $o/ab.txt
}
for r in 1 2 3; do
  for v in base m2 m2s2 m1; do run $v 32 h32_$r --no-roofline --steps 300 --warmup 50; done
done
for r in 1 2; do
  for v in base m2s2; do run $v 256 h256_$r --steps 100 --warmup 30; done
done
