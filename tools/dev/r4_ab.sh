#!/bin/bash
# GPU box (round 4 dev): the Lie tests, then interleaved A/B of build_var/<a> vs build_var/<b> at
# H = 32 and 256, and a kernel trace of variant b at H = 32. Output: gpurun_out/r4/ab/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
a=${1:-base}; b=${2:-poll}; reps=${3:-3}
o=gpurun_out/r4/ab; rm -rf $o; mkdir -p $o
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lie.py -q -m gpu --timeout 120 --timeout-method thread > $o/lie.txt 2>&1; echo "lie rc=$? $(tail -1 $o/lie.txt)"
for H in 32 256; do
  bash tools/dev/ab_run.sh $reps $H fl-slam_amd/build_var/$a/libgcslam.so fl-slam_amd/build_var/$b/libgcslam.so > $o/ab_h$H.txt 2>&1 || { echo "ab H=$H failed"; cat $o/ab_h$H.txt; exit 1; }
  cat $o/ab_h$H.txt
done
d=$o/kt_h32
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o kt --output-format csv -- python3 tools/dev/ab_bench.py fl-slam_amd/build_var/$b/libgcslam.so --hyps 32 --no-cpu --no-roofline --no-map --no-c5 --no-extras --steps 50 --warmup 20 > $d.json 2> $d.err || exit 1
python3 tools/timeline.py "$(find $d -name '*kernel_trace.csv' | head -1)" 14 > $o/timeline_h32.txt
cat $o/timeline_h32.txt
