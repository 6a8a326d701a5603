#!/bin/bash
# GPU box (round 6 dev): the -m gpu suite (SUITE=0 skips it), per-phase cycles at H = 32 (timing build
# fl-slam_amd/ab/timing), then an interleaved A/B of the in-tree library against fl-slam_amd/ab/<variant>
# at H = 32 and H = 256 (bench step, ingest on). Usage: bash tools/dev/r6_ab.sh <tag> <variant> [rounds]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; v=${2:-base}; R=${3:-3}
o=gpurun_out/r6/$tag; rm -rf $o; mkdir -p $o
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
  tail -1 $o/tests.txt
fi
if [ -f fl-slam_amd/ab/timing/libgcslam.so ]; then
  GC_TIMING_LIB=fl-slam_amd/ab/timing/libgcslam.so timeout -k 10 120 python3 tools/phase_timing.py 32 > $o/phases_h32.txt 2>&1 || { tail -5 $o/phases_h32.txt; exit 1; }
fi
stop() { case $1 in 0) ;; *) echo "stopped rc=$1" >> $o/ab.txt; cat $o/ab.txt; tail -5 $o/err.txt; exit $1;; esac; }
run() {  # lib tag H steps warmup
  timeout -k 10 180 python3 tools/dev/ab_bench.py $1 --hyps $3 --no-cpu --no-map --no-c5 --no-roofline --no-dropin --no-extras --steps $4 --warmup $5 > $o/$2.json 2>>$o/err.txt; stop $?
  echo "$2 H=$3 $(tail -1 $o/$2.json | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],4))")" >> $o/ab.txt
}
for r in $(seq 1 $R); do
  run fl-slam_amd/gcslam/libgcslam.so new_h32_$r 32 400 50
  run fl-slam_amd/ab/$v/libgcslam.so ${v}_h32_$r 32 400 50
done
for r in $(seq 1 $R); do
  run fl-slam_amd/gcslam/libgcslam.so new_h256_$r 256 100 30
  run fl-slam_amd/ab/$v/libgcslam.so ${v}_h256_$r 256 100 30
done
cat $o/ab.txt
