#!/bin/bash
# Dev (GPU box): interleaved bench steps of the in-tree library and fl-slam_amd/build_var/<v> for each
# variant given. Usage: bash tools/dev/ab_multi.sh <H> <steps> <rounds> <variant>...
cd "$GRAFT_REPO_ROOT"
H=$1; S=$2; R=$3; shift 3
o=gpurun_out/abm_h$H; rm -rf $o; mkdir -p $o
stop() { case $1 in 124|134|137|139) echo "stopped rc=$1" >> $o/ab.txt; exit $1;; esac; }
for r in $(seq 1 $R); do
  for v in base "$@"; do
    L=fl-slam_amd/build_var/$v/libgcslam.so; [ $v = base ] && L=fl-slam_amd/gcslam/libgcslam.so
    timeout -k 10 180 python3 tools/dev/ab_bench.py $L --hyps $H --no-cpu --no-map --no-c5 --no-roofline --steps $S --warmup 30 > $o/${v}_$r.json 2>>$o/err.txt; stop $?
    echo "$v H=$H $(tail -1 $o/${v}_$r.json | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],4))")" >> $o/ab.txt
  done
done
cat $o/ab.txt
