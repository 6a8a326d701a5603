#!/bin/bash
# GPU box (round 4 dev): C5 in-scan map update kernels per build_var variant (rocprofv3 kernel stats of
# the C5 leg), twice each, interleaved. Usage: bash tools/dev/r4_smap_ab.sh "v1 v2"   Output: gpurun_out/r4/smap_ab/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
vs=$1
o=gpurun_out/r4/smap_ab; rm -rf $o; mkdir -p $o
for r in 1 2; do
  for v in $vs; do
    d=$o/${v}_$r
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o kt --output-format csv -- python3 tools/dev/ab_bench.py fl-slam_amd/build_var/$v/libgcslam.so --c5-only > $d.json 2> $d.err || exit 1
    f=$(find $d -name '*kernel_stats.csv' | head -1)
    python3 - "$f" "$v" "$r" <<'PY' | tee -a $o/ab.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r["Name"]
    if "smap" in n or "fuse" in n:
        out.append("%s avg %.2f us calls %s" % (n.split("(")[0][-22:], float(r["AverageNs"]) / 1e3, r["Calls"]))
print("rep %s %s: %s" % (sys.argv[3], sys.argv[2], "; ".join(out)))
PY
  done
done
