#!/bin/bash
# GPU box (round 4 dev): the -m gpu suite (no -x), an interleaved A/B of build_var/<a> vs <b>, and
# a kernel trace of the C5 legs. Output: gpurun_out/r4/check/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
a=${1:-base}; b=${2:-tail}; reps=${3:-3}
o=gpurun_out/r4/check; rm -rf $o; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $o/gpu_tests.txt 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $o/gpu_tests.txt)"
case $rc in 0|1) ;; *) exit $rc;; esac
for H in 32 256; do
  bash tools/dev/ab_run.sh $reps $H fl-slam_amd/build_var/$a/libgcslam.so fl-slam_amd/build_var/$b/libgcslam.so > $o/ab_h$H.txt 2>&1 || { cat $o/ab_h$H.txt; exit 1; }
  cat $o/ab_h$H.txt
done
d=$o/kt_c5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o kt --output-format csv -- python3 bench.py --c5-only > $d.json 2> $d.err || exit 1
cp "$(find $d -name '*kernel_stats.csv' | head -1)" $o/kernel_stats_c5.csv
find $d -name '*kernel_trace.csv' -delete
tail -c 600 $d.json
