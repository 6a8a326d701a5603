#!/bin/bash
# GPU box (round 5 dev): map tests (staged fuse apply v2: prefetched records, unrolled staging), the
# H = 32 per-wave cycles, the fuse A/B against build_var/unstaged and the fuse PMC passes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s16; rm -rf $o; mkdir -p $o
rc=0; timeout -k 10 300 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread -k "map" > $o/gpu_tests.log 2>&1 || rc=$?
tail -3 $o/gpu_tests.log
case $rc in 0) ;; *) grep -E "Error|assert|FAIL|^E " $o/gpu_tests.log | head -30; echo "gpu tests rc=$rc"; exit $rc;; esac
timeout -k 10 120 python3 tools/phase_timing.py 32 > $o/phases.txt 2>&1 || { tail -5 $o/phases.txt; exit 1; }
cat $o/phases.txt
for i in 1 2 3; do
  for v in staged unstaged; do
    lib=fl-slam_amd/gcslam/libgcslam.so; [ $v = unstaged ] && lib=fl-slam_amd/build_var/unstaged/libgcslam.so
    timeout -k 10 120 python3 tools/dev/ab_bench.py $lib --map-only > $o/fuse_$v.$i.json 2> $o/fuse_$v.$i.err || { tail -5 $o/fuse_$v.$i.err; exit 1; }
    echo "$v $i $(grep -o '"c5_map_fuse": {[^}]*' $o/fuse_$v.$i.json | grep -o '"ms": [0-9.]*')"
  done
done | tee $o/ab_fuse.txt
bash tools/pmc_fuse.sh r05b > $o/pmc_fuse.log 2>&1 || { tail -5 $o/pmc_fuse.log; exit 1; }
tail -12 $o/pmc_fuse.log
