#!/bin/bash
# GPU box (round 5 dev): map tests and the fuse PMC passes after the sector-aligned colour fields and the
# coalesced run-hash wipe, then the fuse A/B against build_var/unstaged256 (the round's previous form).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s19; rm -rf $o; mkdir -p $o
rc=0; timeout -k 10 300 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread -k "map or abi" > $o/gpu_tests.log 2>&1 || rc=$?
tail -3 $o/gpu_tests.log
case $rc in 0) ;; *) grep -E "Error|assert|FAIL|^E " $o/gpu_tests.log | head -30; echo "gpu tests rc=$rc"; exit $rc;; esac
bash tools/pmc_fuse.sh r05 > $o/pmc_fuse.log 2>&1 || { tail -5 $o/pmc_fuse.log; exit 1; }
tail -9 $o/pmc_fuse.log
cp gpurun_out/pmc_fuse_r05.json $o/ 2>/dev/null
for i in 1 2 3; do
  for v in new unstaged256; do
    lib=fl-slam_amd/gcslam/libgcslam.so; [ $v != new ] && lib=fl-slam_amd/build_var/$v/libgcslam.so
    timeout -k 10 120 python3 tools/dev/ab_bench.py $lib --map-only > $o/fuse_$v.$i.json 2> $o/fuse_$v.$i.err || { tail -5 $o/fuse_$v.$i.err; exit 1; }
    echo "$v $i $(grep -o '"c5_map_fuse": {[^}]*' $o/fuse_$v.$i.json | grep -o '"ms": [0-9.]*')"
  done
done | tee $o/ab_fuse.txt
