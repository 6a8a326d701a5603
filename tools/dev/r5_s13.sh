#!/bin/bash
# GPU box (round 5 dev): the -m gpu suite on the in-tree library (stops at the first failure).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-s13}
o=gpurun_out/r5$tag; rm -rf $o; mkdir -p $o
rc=0; timeout -k 10 500 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $o/gpu_tests.log 2>&1 || rc=$?
tail -3 $o/gpu_tests.log
case $rc in 0) ;; *) grep -E "Error|assert|FAIL|^E " $o/gpu_tests.log | head -40; echo "gpu tests rc=$rc"; exit $rc;; esac
