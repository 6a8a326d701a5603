#!/bin/bash
# GPU box (round 5 dev): the -m gpu suite with the short tier at three quarters of a long task per puller for H = 128
# (in-tree), then interleaved A/B against build_var/prev at H = 128, 256 and 32.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s42; rm -rf $o; mkdir -p $o
rc=0; timeout -k 10 500 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || rc=$?
tail -2 $o/gpu_tests.log
case $rc in 0) ;; *) grep -E "Error|assert|FAIL|^E " $o/gpu_tests.log | head -30; echo "gpu tests rc=$rc"; exit $rc;; esac
ab() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  timeout -k 10 180 python3 tools/dev/ab_bench.py $lib --no-cpu --no-map --no-c5 --no-roofline --no-dropin --no-extras "$@" > $o/$tag.json 2>> $o/err.txt || { tail -5 $o/err.txt; exit 1; }
  echo "$tag $(tail -1 $o/$tag.json | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],4))")"
}
for i in 1 2 3; do
  ab new_h128_$i fl-slam_amd/gcslam/libgcslam.so --hyps 128 --steps 200 --warmup 50
  ab prev_h128_$i fl-slam_amd/build_var/prev/libgcslam.so --hyps 128 --steps 200 --warmup 50
  ab new_h256_$i fl-slam_amd/gcslam/libgcslam.so --steps 100 --warmup 30
  ab prev_h256_$i fl-slam_amd/build_var/prev/libgcslam.so --steps 100 --warmup 30
done | tee $o/ab.txt
