#!/bin/bash
# GPU box (round 5 dev): the slot staging's completion-event period against the slot count, interleaved
# at H = 32 and H = 256 (in-tree = every scan's combine_final carries the event; build_var/bindK = every
# K-th scan's).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s20; rm -rf $o; mkdir -p $o
ab() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  timeout -k 10 180 python3 tools/dev/ab_bench.py $lib --no-cpu --no-map --no-c5 --no-roofline --no-dropin --no-extras "$@" > $o/$tag.json 2>> $o/err.txt || { tail -5 $o/err.txt; exit 1; }
  echo "$tag $(tail -1 $o/$tag.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), 'host max/mean', round(d['run_scan_host_ms']['max'],3), round(d['run_scan_host_ms']['mean'],3))")"
}
for i in 1 2 3; do
  ab bind1_s3_h32_$i fl-slam_amd/gcslam/libgcslam.so --hyps 32 --steps 400 --warmup 50
  ab bind1_s4_h32_$i fl-slam_amd/gcslam/libgcslam.so --hyps 32 --steps 400 --warmup 50 --ingest-slots 4
  ab bind2_s4_h32_$i fl-slam_amd/build_var/bind2/libgcslam.so --hyps 32 --steps 400 --warmup 50 --ingest-slots 4
  ab bind2_s5_h32_$i fl-slam_amd/build_var/bind2/libgcslam.so --hyps 32 --steps 400 --warmup 50 --ingest-slots 5
  ab bind3_s6_h32_$i fl-slam_amd/build_var/bind3/libgcslam.so --hyps 32 --steps 400 --warmup 50 --ingest-slots 6
done | tee $o/ab_h32.txt
for i in 1 2; do
  ab bind1_s3_h256_$i fl-slam_amd/gcslam/libgcslam.so --steps 100 --warmup 30
  ab bind2_s4_h256_$i fl-slam_amd/build_var/bind2/libgcslam.so --steps 100 --warmup 30 --ingest-slots 4
  ab bind2_s5_h256_$i fl-slam_amd/build_var/bind2/libgcslam.so --steps 100 --warmup 30 --ingest-slots 5
done | tee $o/ab_h256.txt
