"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch). Dev helper for tools/pmc.sh."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"].split("(")[0][:60]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    if not any(s in k for s in ("soft_assign", "moment_partials", "bins_fused", "evidence", "predict", "combine", "finalize", "k_read", "k_store")):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
