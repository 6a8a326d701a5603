#!/bin/bash
# GPU box (round 4 dev): soft-assign store kinds (sk0 nt, sk1 plain, sk2 sc1) on the contract pair,
# then sacur (before the chain-occupancy / fold changes) vs sk0 at H = 256 and 32.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4/ab3; rm -rf $o; mkdir -p $o
bash tools/dev/r4_saprobe.sh 2 sk0 sk1 sk2 && cp gpurun_out/r4/saprobe/ab.txt $o/saprobe.txt || exit 1
for H in 256 32; do
  bash tools/dev/ab_run.sh 3 $H fl-slam_amd/build_var/sacur/libgcslam.so fl-slam_amd/build_var/sk0/libgcslam.so > $o/ab_h$H.txt 2>&1 || { cat $o/ab_h$H.txt; exit 1; }
  cat $o/ab_h$H.txt
done
