#!/bin/bash
# Dev (GPU box): interleaved A/B of the contract pair (bench.py --roofline-only) between the in-tree
# library and fl-slam_amd/build_var/<variant>. Usage: bash tools/dev/ab_roof.sh <variant> [rounds]
cd "$GRAFT_REPO_ROOT"
v=${1:-base}; R=${2:-3}
o=gpurun_out/abroof_$v; rm -rf $o; mkdir -p $o
stop() { case $1 in 124|134|137|139) echo "stopped rc=$1" >> $o/ab.txt; exit $1;; esac; }
run() {  # lib tag
  timeout -k 10 120 python3 tools/dev/ab_bench.py $1 --roofline-only --roofline-reps 10 > $o/$2.json 2>>$o/err.txt; stop $?
  echo "$2 $(tail -1 $o/$2.json | python3 -c "import json,sys; r=json.loads(sys.stdin.read())['roofline']; p=r['per_kernel']; print(round(r['frac'],4), round(p['soft_assign']['ms'],4), round(p['moment_match']['ms'],4))")" >> $o/ab.txt
}
for r in $(seq 1 $R); do
  run fl-slam_amd/gcslam/libgcslam.so new_$r
  run fl-slam_amd/build_var/$v/libgcslam.so ${v}_$r
done
cat $o/ab.txt
