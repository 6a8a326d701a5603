#!/bin/bash
# GPU box (round 5 dev): the map / scan-map tests, then the C5 map PMC traffic and kernel times
# (tools/pmc_fuse.sh) and the map-only fuse leg.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-s9}
o=gpurun_out/r5$tag; rm -rf $o; mkdir -p $o
rc=0; timeout -k 10 300 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread -k "${PYTEST_K:-map}" > $o/gpu_tests.log 2>&1 || rc=$?
tail -3 $o/gpu_tests.log
case $rc in 0) ;; *) grep -E "Error|assert|FAIL" $o/gpu_tests.log | head -20; echo "gpu tests rc=$rc"; exit $rc;; esac
timeout -k 10 120 python3 bench.py --map-only > $o/map_only.json 2> $o/map_only.err || exit 1
cat $o/map_only.json
bash tools/pmc_fuse.sh r05 > $o/pmc_fuse.log 2>&1 || { tail -5 $o/pmc_fuse.log; exit 1; }
tail -30 $o/pmc_fuse.log
