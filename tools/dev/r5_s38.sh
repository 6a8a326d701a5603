#!/bin/bash
# GPU box (round 5 dev): the bins tiers at H = 256 (32-iteration long tasks, 16-iteration short, 4-iteration tiny),
# interleaved: in-tree against build_var/sd4 (short tasks of 8 iterations, tiny of 2), tp2 (two tiny tasks per
# puller) and td2 (tiny tasks of 8 iterations).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s38; rm -rf $o; mkdir -p $o
ab() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  timeout -k 10 180 python3 tools/dev/ab_bench.py $lib --no-cpu --no-map --no-c5 --no-roofline --no-dropin --no-extras "$@" > $o/$tag.json 2>> $o/err.txt || { tail -5 $o/err.txt; exit 1; }
  echo "$tag $(tail -1 $o/$tag.json | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],4))")"
}
for i in 1 2 3; do
  ab new_$i fl-slam_amd/gcslam/libgcslam.so --steps 100 --warmup 30
  for v in sd4 tp2 td2; do ab ${v}_$i fl-slam_amd/build_var/$v/libgcslam.so --steps 100 --warmup 30; done
done | tee $o/ab.txt
