#!/bin/bash
# GPU box (round 5, session 1): the -m gpu suite (fail-fast tests included), the write-ceiling probe
# (plain / non-temporal streaming writes of 6.4 GB, tools/probe/probe_bw.hip) in the same session as
# the contract pair (bench.py --roofline-only), then the H = 32 shard's kernel timeline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s1; rm -rf $o; mkdir -p $o
rc=0; timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || rc=$?
tail -3 $o/gpu_tests.log
case $rc in 124|134|137|139) echo "gpu tests stopped rc=$rc"; exit $rc;; esac
timeout -k 10 120 ./tools/probe/probe_bw > $o/probe_bw.txt 2>&1 || exit 1
cat $o/probe_bw.txt
timeout -k 10 200 python3 bench.py --roofline-only > $o/roofline.json 2> $o/roofline.err || exit 1
python3 -c "import json;d=json.load(open('$o/roofline.json'))['roofline'];print(d['frac'],d['per_kernel'])"
timeout -k 10 120 ./tools/probe/probe_bw > $o/probe_bw_after.txt 2>&1 || exit 1
bash tools/trace_scan.sh 32 h32 > /dev/null && cp gpurun_out/trace_h32/timeline.txt $o/timeline_h32.txt
cat $o/timeline_h32.txt
