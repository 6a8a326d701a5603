#!/bin/bash
# GPU box (round 4 dev): interleaved A/B of the C5 fuse (c5_map_fuse ms) across build_var variants.
# Usage: bash tools/dev/r4_fuse_ab.sh reps "v1 v2 ..."   Output: gpurun_out/r4/fuse_ab/ab.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
reps=$1; vs=$2
o=gpurun_out/r4/fuse_ab; rm -rf $o; mkdir -p $o
for r in $(seq $reps); do
  for v in $vs; do
    timeout -k 10 120 python3 tools/dev/ab_bench.py fl-slam_amd/build_var/$v/libgcslam.so --map-only > $o/map_${v}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; m=json.loads(open('$o/map_${v}_$r.json').read().strip().splitlines()[-1])['c5_map_fuse']; print('rep $r $v fuse %.4f ms %.0f GB/s distinct %d' % (m['ms'], m['GB/s'], m['distinct_slots']))" | tee -a $o/ab.txt
  done
done
