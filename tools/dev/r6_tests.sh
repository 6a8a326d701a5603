#!/bin/bash
# GPU box (round 6): the -m gpu suite (optionally a -k selection) into gpurun_out/r6/<tag>. Stops after a fault.
cd "$GRAFT_REPO_ROOT"
tag=${1:-all}; sel=${2:-}; xf=${XF--x}
o=gpurun_out/r6/$tag; rm -rf $o; mkdir -p $o
if [ -n "$sel" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu $xf -v --timeout 300 --timeout-method thread -k "$sel" > $o/gpu_tests.txt 2>&1; rc=$?
else
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu $xf -v --timeout 300 --timeout-method thread > $o/gpu_tests.txt 2>&1; rc=$?
fi
echo "tests rc=$rc $(tail -1 $o/gpu_tests.txt)"
exit $rc
