#!/bin/bash
# GPU box (round 4 dev): map / C5 / fuse tests on the in-tree library, then the fuse PMC passes.
# Output: gpurun_out/r4/map_check/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4/map_check; rm -rf $o; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "map or c5 or fuse or scanmap" > $o/tests.txt 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $o/tests.txt)"
[ $rc -eq 0 ] || exit $rc
bash tools/pmc_fuse.sh r04x > $o/pmc_fuse.log 2>&1 || exit 1
cp gpurun_out/pmc_fuse_r04x.json $o/pmc_fuse.json; rm -rf gpurun_out/pmc_fuse
tail -8 $o/pmc_fuse.log
