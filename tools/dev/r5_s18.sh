#!/bin/bash
# GPU box (round 5 dev): the -m gpu suite, the fuse PMC passes (staged apply, 256-row sort blocks), the
# fuse A/B against build_var/unstaged256 and build_var/unstaged (512), the H = 32 chain cycles and the
# H = 32 A/B against build_var/ev1 (predict's dt_imu moved to wave 3).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s18; rm -rf $o; mkdir -p $o
rc=0; timeout -k 10 500 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || rc=$?
tail -3 $o/gpu_tests.log
case $rc in 0) ;; *) grep -E "Error|assert|FAIL|^E " $o/gpu_tests.log | head -30; echo "gpu tests rc=$rc"; exit $rc;; esac
bash tools/pmc_fuse.sh r05 > $o/pmc_fuse.log 2>&1 || { tail -5 $o/pmc_fuse.log; exit 1; }
tail -9 $o/pmc_fuse.log
for i in 1 2; do
  for v in staged256 unstaged256 unstaged; do
    lib=fl-slam_amd/gcslam/libgcslam.so; [ $v != staged256 ] && lib=fl-slam_amd/build_var/$v/libgcslam.so
    timeout -k 10 120 python3 tools/dev/ab_bench.py $lib --map-only > $o/fuse_$v.$i.json 2> $o/fuse_$v.$i.err || { tail -5 $o/fuse_$v.$i.err; exit 1; }
    echo "$v $i $(grep -o '"c5_map_fuse": {[^}]*' $o/fuse_$v.$i.json | grep -o '"ms": [0-9.]*')"
  done
done | tee $o/ab_fuse.txt
timeout -k 10 120 python3 tools/phase_timing.py 32 > $o/phases.txt 2>&1 || { tail -5 $o/phases.txt; exit 1; }
grep -E "predict: (Σ|lift|pose0|loads|moments)|predict total" $o/phases.txt
ab() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  timeout -k 10 180 python3 tools/dev/ab_bench.py $lib --no-cpu --no-map --no-c5 --no-roofline --no-dropin "$@" > $o/$tag.json 2>> $o/err.txt || { tail -5 $o/err.txt; exit 1; }
  echo "$tag $(tail -1 $o/$tag.json | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],4))")"
}
for i in 1 2 3; do
  ab new_h32_$i fl-slam_amd/gcslam/libgcslam.so --hyps 32 --steps 400 --warmup 50
  ab ev1_h32_$i fl-slam_amd/build_var/ev1/libgcslam.so --hyps 32 --steps 400 --warmup 50
done | tee $o/ab_h32.txt
