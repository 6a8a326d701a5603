#!/bin/bash
# GPU box (round 6 dev): interleaved A/B of several arms at H = 32 and H = 256 (bench step, ingest on),
# each arm a library and extra bench arguments. Usage:
#   bash tools/dev/r6_abn.sh <tag> <rounds> "<label>|<lib>|<bench args>" ...
# e.g. "base|fl-slam_amd/gcslam/libgcslam.so|" "bind2s4|fl-slam_amd/ab/bind2/libgcslam.so|--ingest-slots 4"
# Output: gpurun_out/r6/<tag>/ab.txt (one line per run: label, H, ms per step). Stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; R=$2; shift 2
o=gpurun_out/r6/$tag; rm -rf $o; mkdir -p $o
run() {  # label lib H steps warmup args
  timeout -k 10 180 python3 tools/dev/ab_bench.py $2 --hyps $3 --no-cpu --no-map --no-c5 --no-roofline --no-dropin --no-extras \
    --steps $4 --warmup $5 $6 > $o/$1_h$3.json 2>>$o/err.txt || { echo "stopped: $1 H=$3" >> $o/ab.txt; cat $o/ab.txt; tail -5 $o/err.txt; exit 1; }
  echo "$1 H=$3 $(tail -1 $o/$1_h$3.json | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],4))")" >> $o/ab.txt
}
for H in 32 256; do
  st=400; wu=50; [ $H = 256 ] && st=100 && wu=30
  for r in $(seq 1 $R); do
    for arm in "$@"; do
      IFS='|' read -r label lib args <<< "$arm"
      run $label $lib $H $st $wu "$args"
    done
  done
done
cat $o/ab.txt
