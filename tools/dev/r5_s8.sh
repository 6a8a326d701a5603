#!/bin/bash
# GPU box (round 5 dev): the -m gpu suite, the H = 32 / H = 256 steps, the H = 32 timeline, the chain
# kernels' phase cycles.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-s8}
o=gpurun_out/r5$tag; rm -rf $o; mkdir -p $o
rc=0; timeout -k 10 500 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $o/gpu_tests.log 2>&1 || rc=$?
tail -3 $o/gpu_tests.log
case $rc in 0) ;; *) grep -E "Error|assert|FAIL" $o/gpu_tests.log | head -20; echo "gpu tests rc=$rc"; exit $rc;; esac
timeout -k 10 200 python3 bench.py --hyps 32 --steps 400 --warmup 50 --no-cpu --no-roofline --no-map --no-c5 --no-dropin > $o/bench_h32.json 2> $o/bench_h32.err || exit 1
python3 tools/summ.py $o/bench_h32.json
timeout -k 10 200 python3 bench.py --steps 100 --warmup 50 --no-cpu --no-roofline --no-map --no-c5 --no-dropin > $o/bench.json 2> $o/bench.err || exit 1
python3 tools/summ.py $o/bench.json
bash tools/trace_scan.sh 32 h32 > /dev/null && python3 tools/timeline.py "$(find gpurun_out/trace_h32/kt -name '*kernel_trace.csv' | head -1)" 40 > $o/timeline_h32_long.txt && tail -14 $o/timeline_h32_long.txt
timeout -k 10 120 python3 tools/phase_timing.py 32 > $o/phases.txt 2>&1; grep -E "predict:|evidence: (start|MF\.\.|L_raw|pose6|fusion|recompose|IW|map inc|drift)|total" $o/phases.txt
