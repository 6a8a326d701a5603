#!/bin/bash
# GPU box (round 4 dev): interleaved A/B of (library variant, ingest slots) pairs at H = 32 and 256.
# Usage: bash tools/dev/r4_ab_slots.sh reps "base:3 poll:4 base:4"   Output: gpurun_out/r4/ab_slots/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
reps=$1; shift; cfgs=$1
o=gpurun_out/r4/ab_slots; rm -rf $o; mkdir -p $o
for H in ${HS:-32 256}; do
  for r in $(seq $reps); do
    for c in $cfgs; do
      v=${c%%:*}; sl=${c##*:}
      ms=$(timeout -k 10 120 python3 tools/dev/ab_bench.py fl-slam_amd/build_var/$v/libgcslam.so --hyps $H --ingest-slots $sl --no-cpu --no-roofline --no-map --no-c5 --no-extras --steps 300 --warmup 100 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('%.4f host_max %.3f mean %.3f' % (d['ms_per_step'], d['run_scan_host_ms']['max'], d['run_scan_host_ms']['mean']))") || exit 1
      echo "rep $r H=$H $v slots=$sl $ms" | tee -a $o/ab.txt
    done
  done
done
