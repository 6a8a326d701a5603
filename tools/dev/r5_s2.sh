#!/bin/bash
# GPU box (round 5 dev): the -m gpu suite on the in-tree library, then the H = 32 shard and the C3
# step (bench lines without the extra legs), then the H = 32 kernel timeline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-s2}
o=gpurun_out/r5$tag; rm -rf $o; mkdir -p $o
rc=0; timeout -k 10 500 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $o/gpu_tests.log 2>&1 || rc=$?
tail -15 $o/gpu_tests.log
case $rc in 0) ;; *) echo "gpu tests rc=$rc"; exit $rc;; esac
timeout -k 10 200 python3 bench.py --hyps 32 --steps 400 --warmup 50 --no-cpu --no-roofline --no-map --no-c5 --no-dropin > $o/bench_h32.json 2> $o/bench_h32.err || exit 1
python3 tools/summ.py $o/bench_h32.json
timeout -k 10 200 python3 bench.py --steps 100 --warmup 50 --no-cpu --no-roofline --no-map --no-c5 --no-dropin > $o/bench.json 2> $o/bench.err || exit 1
python3 tools/summ.py $o/bench.json
bash tools/trace_scan.sh 32 h32 > /dev/null && cp gpurun_out/trace_h32/timeline.txt $o/timeline_h32.txt && tail -8 $o/timeline_h32.txt
