#!/bin/bash
# GPU box (round 4 dev): map tests, the C5 fuse of build_var/noxcd vs xcd (interleaved), and the
# fuse PMC passes on the in-tree library. Output: gpurun_out/r4/xcd/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4/xcd; rm -rf $o; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "map or c5 or fuse or scanmap" > $o/tests.txt 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $o/tests.txt)"
case $rc in 0|1) ;; *) exit $rc;; esac
for r in 1 2 3; do
  for v in noxcd xcd; do
    timeout -k 10 120 python3 tools/dev/ab_bench.py fl-slam_amd/build_var/$v/libgcslam.so --map-only > $o/map_${v}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; m=json.loads(open('$o/map_${v}_$r.json').read().strip().splitlines()[-1])['c5_map_fuse']; print('rep $r $v fuse %.4f ms %.0f GB/s' % (m['ms'], m['GB/s']))" | tee -a $o/ab.txt
  done
done
bash tools/pmc_fuse.sh r04x > $o/pmc_fuse.log 2>&1 || exit 1
cp gpurun_out/pmc_fuse_r04x.json $o/pmc_fuse.json; rm -rf gpurun_out/pmc_fuse
tail -8 $o/pmc_fuse.log
