#!/bin/bash
# GPU box (round 5 dev): map / scan-map tests on the in-tree library (the staged fuse apply), the H = 32
# chain's per-phase / per-wave cycles, an interleaved A/B of the standalone C5 fuse (in-tree vs
# build_var/unstaged), the fuse PMC passes, and an interleaved H = 32 A/B of build_var/fin32.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s15; rm -rf $o; mkdir -p $o
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
tail -40 $o/pmc_fuse.log
for i in 1 2 3; do
  for v in base fin32; do
    lib=fl-slam_amd/gcslam/libgcslam.so; [ $v = fin32 ] && lib=fl-slam_amd/build_var/fin32/libgcslam.so
    timeout -k 10 180 python3 tools/dev/ab_bench.py $lib --hyps 32 --no-cpu --no-map --no-c5 --no-roofline --no-dropin --steps 400 --warmup 50 > $o/h32_$v.$i.json 2>> $o/h32_err.txt || { tail -5 $o/h32_err.txt; exit 1; }
    echo "$v $i $(tail -1 $o/h32_$v.$i.json | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],4))")"
  done
done | tee $o/ab_fin32.txt
