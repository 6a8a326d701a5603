#!/bin/bash
# GPU box (round 5 dev): A/B of the in-scan map update on its own stream (default build) against the
# compute stream (build_var/smap0, -DGC_SMAP_SIDE=0), C5 legs alternated three times.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s11; rm -rf $o; mkdir -p $o
for i in 1 2 3; do
  for v in side smap0; do
    lib=fl-slam_amd/gcslam/libgcslam.so; [ $v = smap0 ] && lib=fl-slam_amd/build_var/smap0/libgcslam.so
    timeout -k 10 200 python3 tools/dev/ab_bench.py $lib --c5-only > $o/$v.$i.json 2> $o/$v.$i.err || { tail -5 $o/$v.$i.err; exit 1; }
    echo "$v $i $(grep -o '"c5": {[^}]*' $o/$v.$i.json | grep -o 'ms_per_scan": [0-9.]*') $(grep -o '"c5_dense": {[^}]*' $o/$v.$i.json | grep -o 'ms_per_scan": [0-9.]*')"
  done
done | tee $o/ab.txt
