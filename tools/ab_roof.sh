#!/bin/bash
# Dev (GPU box): interleaved A/B of the contract pair (bench.py --roofline-only) across library builds.
# Usage: bash tools/ab_roof.sh <reps> <lib1> <lib2> ...
reps=$1; shift
for r in $(seq $reps); do
  for lib in "$@"; do
    mkdir -p gpurun_out; out=$(timeout -k 10 120 python3 tools/ab_bench.py $lib --roofline-only 2>gpurun_out/ab_roof.err) || { tail -5 gpurun_out/ab_roof.err; exit 1; }
    echo "$out" | python3 -c "import json,sys; r=json.loads(sys.stdin.read().strip().splitlines()[-1])['roofline']; pk=r['per_kernel']; print('rep $r $lib sa %.4f ms %.0f GB/s  mm %.4f ms %.0f GB/s  frac %.3f' % (pk['soft_assign']['ms'], pk['soft_assign']['GB/s'], pk['moment_match']['ms'], pk['moment_match']['GB/s'], r['frac']))"
  done
done
