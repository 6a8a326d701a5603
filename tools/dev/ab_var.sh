#!/bin/bash
# Dev (GPU box): interleaved A/B of the in-tree library against fl-slam_amd/build_var/<variant> at
# H = 32 and H = 256 (bench step, ingest on). Usage: bash tools/dev/ab_var.sh <variant> [rounds]
cd "$GRAFT_REPO_ROOT"
v=${1:-base}; R=${2:-3}
o=gpurun_out/ab_$v; rm -rf $o; mkdir -p $o
stop() { case $1 in 124|134|137|139) echo "stopped rc=$1" >> $o/ab.txt; exit $1;; esac; }
run() {  # lib tag H steps warmup
  timeout -k 10 180 python3 tools/dev/ab_bench.py $1 --hyps $3 --no-cpu --no-map --no-c5 --no-roofline --steps $4 --warmup $5 > $o/$2.json 2>>$o/err.txt; stop $?
  echo "$2 H=$3 $(tail -1 $o/$2.json | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],4))")" >> $o/ab.txt
}
for r in $(seq 1 $R); do
  run fl-slam_amd/gcslam/libgcslam.so new_h32_$r 32 400 50
  run fl-slam_amd/build_var/$v/libgcslam.so ${v}_h32_$r 32 400 50
done
for r in $(seq 1 $R); do
  run fl-slam_amd/gcslam/libgcslam.so new_h256_$r 256 100 30
  run fl-slam_amd/build_var/$v/libgcslam.so ${v}_h256_$r 256 100 30
done
cat $o/ab.txt
