#!/bin/bash
# GPU box (round 5 dev): the bins tiers around the round's H = 32 setting (short tier half a long task per puller),
# interleaved at H = 32: in-tree against build_var/sd1 (short tasks as long as the long ones), td2 (tiny tasks of
# half a short one), ss04 / ss06 (the short share 0.4 / 0.6) and mt1 (one long task per puller).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s31; rm -rf $o; mkdir -p $o
ab() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  timeout -k 10 180 python3 tools/dev/ab_bench.py $lib --no-cpu --no-map --no-c5 --no-roofline --no-dropin --no-extras "$@" > $o/$tag.json 2>> $o/err.txt || { tail -5 $o/err.txt; exit 1; }
  echo "$tag $(tail -1 $o/$tag.json | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],4))")"
}
for i in 1 2 3; do
  ab new_$i fl-slam_amd/gcslam/libgcslam.so --hyps 32 --steps 400 --warmup 50
  for v in sd1 td2 ss04 ss06 mt1; do ab ${v}_$i fl-slam_amd/build_var/$v/libgcslam.so --hyps 32 --steps 400 --warmup 50; done
done | tee $o/ab.txt
