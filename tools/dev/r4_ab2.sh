#!/bin/bash
# GPU box (round 4 dev): the -m gpu suite on the in-tree library, interleaved A/B of build_var/lb1
# (chain kernels at one workgroup per CU), lb2 (occupancy by grid size) and fold (+ the a6 finalize
# folded into k_evidence) at H = 32 and 256, then the contract pair / fuse probe.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4/ab2; rm -rf $o; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $o/gpu_tests.txt 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $o/gpu_tests.txt)"
case $rc in 0|1) ;; *) exit $rc;; esac
for H in 256 32; do
  bash tools/dev/ab_run.sh 3 $H fl-slam_amd/build_var/lb1/libgcslam.so fl-slam_amd/build_var/lb2/libgcslam.so fl-slam_amd/build_var/fold/libgcslam.so > $o/ab_h$H.txt 2>&1 || { cat $o/ab_h$H.txt; exit 1; }
  cat $o/ab_h$H.txt
done
bash tools/dev/r4_saprobe.sh 2 sacur sastore f512 && cp gpurun_out/r4/saprobe/ab.txt $o/saprobe.txt
