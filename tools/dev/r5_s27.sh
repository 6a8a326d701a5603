#!/bin/bash
# GPU box (round 5 dev): the hand-written device radix sort (gc_sort.hip) in place of the library sorts: its own
# tests against NumPy's stable argsort, then the map maintenance and association tests that use it, then the
# whole -m gpu suite.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s27; rm -rf $o; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py tests/test_map_ops.py tests/test_association.py -x -v -m gpu --timeout 120 --timeout-method thread > $o/sort_tests.log 2>&1 || { tail -40 $o/sort_tests.log; exit 1; }
tail -2 $o/sort_tests.log
timeout -k 10 500 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -2 $o/gpu_tests.log
