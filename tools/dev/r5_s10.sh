#!/bin/bash
# GPU box (round 5 dev): the -m gpu suite, the C5 legs (side-stream map update) with a kernel trace of
# their last scans, then the default bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-s10}
o=gpurun_out/r5$tag; rm -rf $o; mkdir -p $o
rc=0; timeout -k 10 500 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $o/gpu_tests.log 2>&1 || rc=$?
tail -3 $o/gpu_tests.log
case $rc in 0) ;; *) grep -E "Error|assert|FAIL" $o/gpu_tests.log | head -20; echo "gpu tests rc=$rc"; exit $rc;; esac
timeout -k 10 200 rocprofv3 --kernel-trace -d $o/kt -o kt --output-format csv -- python3 bench.py --c5-only > $o/c5.json 2> $o/c5.err || { tail -5 $o/c5.err; exit 1; }
cat $o/c5.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); [print(k, {q: v[q] for q in v if q in ('ms_per_scan','ms','scans_per_s','hyps_per_s')}) for k, v in d.items()]"
python3 tools/timeline.py "$(find $o/kt -name '*kernel_trace.csv' | head -1)" 24 > $o/timeline_c5.txt; tail -24 $o/timeline_c5.txt
timeout -k 10 300 python3 bench.py > $o/bench.json 2> $o/bench.err || { tail -5 $o/bench.err; exit 1; }
python3 tools/summ.py $o/bench.json
