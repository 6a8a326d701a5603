#!/bin/bash
# GPU box (round 5 dev): the bins launch's short tier per puller (GC_BINS_SHORT_SHARE: the short tasks' work as a
# fraction of one long task per puller; in-tree 1.0), interleaved at H = 32 (0.25, 0.35, 0.5, 0.75) and H = 256
# (0.5, 0.75).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s29; rm -rf $o; mkdir -p $o
ab() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  timeout -k 10 180 python3 tools/dev/ab_bench.py $lib --no-cpu --no-map --no-c5 --no-roofline --no-dropin --no-extras "$@" > $o/$tag.json 2>> $o/err.txt || { tail -5 $o/err.txt; exit 1; }
  echo "$tag $(tail -1 $o/$tag.json | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],4))")"
}
for i in 1 2 3; do
  ab new_h32_$i fl-slam_amd/gcslam/libgcslam.so --hyps 32 --steps 400 --warmup 50
  for v in ss025 ss035 ss05 ss075; do ab ${v}_h32_$i fl-slam_amd/build_var/$v/libgcslam.so --hyps 32 --steps 400 --warmup 50; done
  ab new_h256_$i fl-slam_amd/gcslam/libgcslam.so --steps 100 --warmup 30
  for v in ss05 ss075; do ab ${v}_h256_$i fl-slam_amd/build_var/$v/libgcslam.so --steps 100 --warmup 30; done
done | tee $o/ab.txt
