#!/bin/bash
# GPU box (round 4 probe): contract-pair roofline and the standalone C5 fuse of build_var variants
# (interleaved). Usage: bash tools/dev/r4_saprobe.sh reps v1 v2 ...   Output: gpurun_out/r4/saprobe/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
reps=$1; shift
o=gpurun_out/r4/saprobe; rm -rf $o; mkdir -p $o
for r in $(seq $reps); do
  for v in "$@"; do
    timeout -k 10 120 python3 tools/dev/ab_bench.py fl-slam_amd/build_var/$v/libgcslam.so --roofline-only > $o/roof_${v}_${r}.json 2>/dev/null || exit 1
    timeout -k 10 120 python3 tools/dev/ab_bench.py fl-slam_amd/build_var/$v/libgcslam.so --map-only > $o/map_${v}_${r}.json 2>/dev/null || exit 1
    python3 -c "
import json
d=json.loads(open('$o/roof_${v}_${r}.json').read().strip().splitlines()[-1]); r=d['roofline']; pk=r['per_kernel']
m=json.loads(open('$o/map_${v}_${r}.json').read().strip().splitlines()[-1])['c5_map_fuse']
print('rep $r $v frac %.4f sa %.3f ms %.0f GB/s mm %.3f ms | fuse %.4f ms %.0f GB/s' % (r['frac'], pk['soft_assign']['ms'], pk['soft_assign']['GB/s'], pk['moment_match']['ms'], m['ms'], m['GB/s']))" | tee -a $o/ab.txt
  done
done
