#!/bin/bash
# GPU box (round 4 dev): map tests, then the C5 legs under a kernel trace (per-call durations kept)
# and the standalone fuse leg. Output: gpurun_out/r4/map/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4/map; rm -rf $o; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "map or c5 or fuse or scanmap" > $o/tests.txt 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $o/tests.txt)"
case $rc in 0|1) ;; *) exit $rc;; esac
d=$o/kt_c5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o kt --output-format csv -- python3 bench.py --c5-only > $d.json 2> $d.err || exit 1
f=$(find $d -name '*kernel_trace.csv' | head -1)
python3 - "$f" > $o/map_calls.txt <<'PY'
import csv, re, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    n = r["Kernel_Name"]
    if "smap" in n or "fuse" in n:
        m = re.search(r"(k_\w+)", n)
        print("%-24s %8.1f" % (m.group(1) if m else n[:24], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
PY
cp "$(find $d -name '*kernel_stats.csv' | head -1)" $o/kernel_stats_c5.csv
find $d -name '*kernel_trace.csv' -delete
timeout -k 10 200 python3 bench.py --map-only > $o/map_only.json 2> $o/map_only.err || exit 1
tail -c 500 $o/map_only.json
cat $o/map_calls.txt | tail -40
