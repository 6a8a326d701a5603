#!/bin/bash
# GPU box (round 5 dev): the short-tier share at H = 64 (the 4-rank shard of C4: 16-iteration long tasks; in-tree 0.5; the variants were built with a GC_BINS_SHORT_SHARE_16 knob not kept),
# interleaved: in-tree vs build_var/s16a (0.75) and s16b (0.25).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s43; rm -rf $o; mkdir -p $o
ab() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  timeout -k 10 180 python3 tools/dev/ab_bench.py $lib --no-cpu --no-map --no-c5 --no-roofline --no-dropin --no-extras "$@" > $o/$tag.json 2>> $o/err.txt || { tail -5 $o/err.txt; exit 1; }
  echo "$tag $(tail -1 $o/$tag.json | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],4))")"
}
for i in 1 2 3; do
  ab new_h64_$i fl-slam_amd/gcslam/libgcslam.so --hyps 64 --steps 300 --warmup 50
  for v in s16a s16b; do ab ${v}_h64_$i fl-slam_amd/build_var/$v/libgcslam.so --hyps 64 --steps 300 --warmup 50; done
done | tee $o/ab.txt
