#!/bin/bash
# GPU box (round 5 dev): the short-tier share at H = 128 (the 2-rank shard of C4: 32-iteration long tasks, where the
# in-tree rule keeps one long task per puller), interleaved: in-tree vs build_var/all05 (half) and all075 (three quarters).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s41; rm -rf $o; mkdir -p $o
ab() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  timeout -k 10 180 python3 tools/dev/ab_bench.py $lib --no-cpu --no-map --no-c5 --no-roofline --no-dropin --no-extras "$@" > $o/$tag.json 2>> $o/err.txt || { tail -5 $o/err.txt; exit 1; }
  echo "$tag $(tail -1 $o/$tag.json | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],4))")"
}
for i in 1 2 3; do
  ab new_h128_$i fl-slam_amd/gcslam/libgcslam.so --hyps 128 --steps 200 --warmup 50
  for v in all05 all075; do ab ${v}_h128_$i fl-slam_amd/build_var/$v/libgcslam.so --hyps 128 --steps 200 --warmup 50; done
done | tee $o/ab.txt
