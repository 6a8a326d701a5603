#!/bin/bash
# GPU box (round 6 dev): the drop-in tests, the drop-in leg's host profile (cProfile) and a kernel +
# memory-copy trace of bench.py --dropin-only with per-kernel stats.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r6/${1:-dropin}; rm -rf $o; mkdir -p $o
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k dropin > $o/tests.txt 2>&1 || { tail -20 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
timeout -k 10 300 python3 tools/dev/r6_dropin_prof.py $o/prof.txt > $o/prof.log 2>&1 || { tail -5 $o/prof.log; exit 1; }
head -1 $o/prof.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $o/rp -o rp --output-format csv -- python3 bench.py --dropin-only > $o/rp.json 2> $o/rp.err || { tail -5 $o/rp.err; exit 1; }
cat $o/rp.json
f=$(find $o/rp -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:25]:
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.1f} pct={float(r['Percentage']):6.2f}")
PY
f=$(find $o/rp -name "*memory_copy_stats.csv" | head -1); [ -n "$f" ] && cat "$f"
exit 0
