#!/bin/bash
# GPU box (round 5 dev): soft-assign / moment tests on the in-tree library, the contract pair A/B
# (in-tree nt + reversed moment grid vs forward grid, plain and sc1 row stores), the H = 32 timeline
# and the chain kernels' phase cycles.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s7; rm -rf $o; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_points.py -q -x -m gpu --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -20 $o/tests.log; exit 1; }
tail -1 $o/tests.log
stop() { case $1 in 0) ;; *) echo "stopped rc=$1"; exit $1;; esac; }
run() {  # lib tag
  timeout -k 10 120 python3 tools/dev/ab_bench.py $1 --roofline-only --roofline-reps 10 > $o/$2.json 2>>$o/err.txt; stop $?
  echo "$2 $(tail -1 $o/$2.json | python3 -c "import json,sys; r=json.loads(sys.stdin.read())['roofline']; p=r['per_kernel']; print(round(r['frac'],4), round(p['soft_assign']['ms'],4), round(p['moment_match']['ms'],4), round(p['soft_assign']['GB/s']), round(p['moment_match']['GB/s']))")" >> $o/ab.txt
}
for r in 1 2 3; do
  run fl-slam_amd/gcslam/libgcslam.so ntrev_$r
  run fl-slam_amd/build_var/momfwd/libgcslam.so ntfwd_$r
  run fl-slam_amd/build_var/saplain/libgcslam.so plainrev_$r
  run fl-slam_amd/build_var/sasc1/libgcslam.so sc1rev_$r
done
cat $o/ab.txt
timeout -k 10 120 ./tools/probe/probe_bw > $o/probe_bw.txt 2>&1; stop $?
cat $o/probe_bw.txt
bash tools/trace_scan.sh 32 h32 > /dev/null && cp gpurun_out/trace_h32/timeline.txt $o/timeline_h32.txt && python3 tools/timeline.py "$(find gpurun_out/trace_h32/kt -name '*kernel_trace.csv' | head -1)" 40 > $o/timeline_h32_long.txt; tail -16 $o/timeline_h32_long.txt
timeout -k 10 120 python3 tools/phase_timing.py 32 > $o/phases.txt 2>&1; cat $o/phases.txt
