#!/bin/bash
# GPU box (round 5 dev): the C5 fuse's run-hash load factor. PMC bytes (FETCH_SIZE, WRITE_SIZE) and the kernel trace
# of bench.py --map-only for the in-tree library (2^bits >= 4 x rows entries) and build_var/load2 (2 x rows) and
# load1 (1 x rows), then the three interleaved (ms of c5_map_fuse).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5s26; rm -rf $o; mkdir -p $o
for v in base load2 load1; do
  lib=fl-slam_amd/gcslam/libgcslam.so; [ $v = base ] || lib=fl-slam_amd/build_var/$v/libgcslam.so
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $o/$v/fetch -o fetch --output-format csv -- python3 tools/dev/ab_bench.py $lib --map-only > $o/$v.fetch.log 2>&1 || { tail -5 $o/$v.fetch.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $o/$v/write -o write --output-format csv -- python3 tools/dev/ab_bench.py $lib --map-only > $o/$v.write.log 2>&1 || { tail -5 $o/$v.write.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $o/$v/kt -o kt --output-format csv -- python3 tools/dev/ab_bench.py $lib --map-only > $o/$v.kt.log 2>&1 || { tail -5 $o/$v.kt.log; exit 1; }
  echo "pmc $v done"
done
for i in 1 2 3; do
  for v in base load2 load1; do
    lib=fl-slam_amd/gcslam/libgcslam.so; [ $v = base ] || lib=fl-slam_amd/build_var/$v/libgcslam.so
    timeout -k 10 120 python3 tools/dev/ab_bench.py $lib --map-only > $o/t_${v}_$i.json 2>> $o/err.txt || { tail -5 $o/err.txt; exit 1; }
    echo "${v}_$i $(tail -1 $o/t_${v}_$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d["c5_map_fuse"]; print(round(m["ms"],5), m.get("distinct_slots"))")"
  done
done | tee $o/ab.txt
