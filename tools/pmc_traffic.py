"""Summarise the contract pair's PMC passes (tools/pmc_traffic.sh) into pmc_traffic.json.

HBM bytes per launch = 2 x FETCH_SIZE (gfx950: FETCH_SIZE reports half the bytes of wide coalesced
reads, MI355X_MICROARCH.md 'HBM') + WRITE_SIZE, per kernel, averaged over dispatches; the pair is
k_soft_assign + k_soft_assign_finalize + k_moment_partials + k_bins_finalize. The request-size
breakdown (TCC_EA0_RDREQ_{128B,64B,32B}) is kept beside it as a cross-check."""
import collections
import csv
import glob
import json
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
pair = ("k_soft_assign<", "k_soft_assign_finalize", "k_moment_partials<", "k_bins_finalize")
per = {}
total = 0.0
for k, cs in acc.items():
    if not any(p in k for p in pair):
        continue
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    rd = 2.0 * m.get("FETCH_SIZE", 0.0) * 1024
    wr = m.get("WRITE_SIZE", 0.0) * 1024
    sized = 128 * m.get("TCC_EA0_RDREQ_128B", 0) + 64 * m.get("TCC_EA0_RDREQ_64B", 0) + 32 * m.get("TCC_EA0_RDREQ_32B", 0)
    per[k] = {"read_bytes": rd, "write_bytes": wr, "rdreq_sized_bytes": sized,
              "counters": {c: v for c, v in m.items()}, "dispatches": len(next(iter(cs.values())))}
    total += rd + wr
bench = [l for l in open(os.path.join(src, "fetch.log")) if l.startswith("{")]
shape = json.loads(bench[-1])["roofline"] if bench else {}
out = {"pair_bytes": total, "per_kernel": per, "H": shape.get("hypotheses"), "n": shape.get("points"), "B": shape.get("bins"),
       "algorithmic_bytes": sum(v["bytes"] for v in shape.get("per_kernel", {}).values()),
       "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --roofline-only "
                 "(tools/pmc_traffic.sh); read = 2 x FETCH_SIZE (gfx950 correction)"}
os.makedirs(os.path.dirname(dst), exist_ok=True)
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps({k: (round(v["read_bytes"] / 1e9, 3), round(v["write_bytes"] / 1e9, 3),
                      round(v["rdreq_sized_bytes"] / 1e9, 3)) for k, v in per.items()}))
print("pair bytes/launch %.3f GB vs algorithmic %.3f GB" % (total / 1e9, out["algorithmic_bytes"] / 1e9))
