#!/bin/bash
# GPU box (round 5 dev): the H = 32 shard's split finalize, interleaved A/B: in-tree (16 chunk records per
# load batch) against build_var/ku32 and ku64 (32 / 64 per batch: one L2 round trip for H = 32's 62 records)
# and build_var/fold64 (the records folded into k_evidence up to 64 chunks: no split launch at H = 32).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s25; rm -rf $o; mkdir -p $o
ab() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  timeout -k 10 180 python3 tools/dev/ab_bench.py $lib --no-cpu --no-map --no-c5 --no-roofline --no-dropin --no-extras "$@" > $o/$tag.json 2>> $o/err.txt || { tail -5 $o/err.txt; exit 1; }
  echo "$tag $(tail -1 $o/$tag.json | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],4))")"
}
for i in 1 2 3; do
  ab new_$i fl-slam_amd/gcslam/libgcslam.so --hyps 32 --steps 400 --warmup 50
  ab ku32_$i fl-slam_amd/build_var/ku32/libgcslam.so --hyps 32 --steps 400 --warmup 50
  ab ku64_$i fl-slam_amd/build_var/ku64/libgcslam.so --hyps 32 --steps 400 --warmup 50
  ab fold64_$i fl-slam_amd/build_var/fold64/libgcslam.so --hyps 32 --steps 400 --warmup 50
done | tee $o/ab.txt
