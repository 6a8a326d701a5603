#!/bin/bash
# GPU box (round 4 dev): soft-assign tests on the in-tree library, then interleaved contract-pair
# roofline runs of build_var/<a> vs <b>. Output: gpurun_out/r4/sa/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
a=${1:-sa0}; b=${2:-sa1}; reps=${3:-3}
o=gpurun_out/r4/sa; rm -rf $o; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "soft or contract or binning or golden or points" > $o/tests.txt 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $o/tests.txt)"
case $rc in 0|1) ;; *) exit $rc;; esac
for r in $(seq $reps); do
  for v in $a $b; do
    timeout -k 10 120 python3 tools/dev/ab_bench.py fl-slam_amd/build_var/$v/libgcslam.so --roofline-only > $o/roof_${v}_${r}.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('$o/roof_${v}_${r}.json').read().strip().splitlines()[-1]); r=d['roofline']; pk=r['per_kernel']; print('rep $r $v frac %.4f sa %.3f ms %.0f GB/s mm %.3f ms' % (r['frac'], pk['soft_assign']['ms'], pk['soft_assign']['GB/s'], pk['moment_match']['ms']))" | tee -a $o/ab.txt
  done
done
