#!/bin/bash
# Dev (GPU box): interleaved A/B of library variants on the bench step.
# Usage: bash tools/dev/ab_run.sh <reps> <hyps> <lib1> <lib2> ...   (prints ms/scan per run)
reps=$1; hyps=$2; shift 2
for r in $(seq $reps); do
  for lib in "$@"; do
    ms=$(timeout -k 10 120 python3 tools/dev/ab_bench.py $lib --hyps $hyps --no-cpu --no-roofline --no-map --no-c5 --steps 200 --warmup 100 2>/dev/null | python3 -c "import json,sys; print('%.4f' % json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
    echo "rep $r H=$hyps $lib $ms"
  done
done
