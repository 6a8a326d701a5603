"""Summarise tools/pmc_fuse.sh: per C5 map kernel, HBM bytes per dispatch (reads by EA request size,
with 2 x FETCH_SIZE beside it, + WRITE_SIZE) and the average duration from the kernel
trace of the same command; the leg's algorithmic bytes from its bench JSON line."""
import collections
import csv
import glob
import json
import os
import re
import sys


def kname(full):
    """k_* kernel name (anonymous namespaces included), or the rocprim kernel's short name."""
    m = re.search(r"(k_\w+)", full)
    if m:
        return m.group(1)
    m = re.search(r"(\w*(?:sort|Sort|onesweep|histogram|scan)\w*)", full)
    return ("rocprim:" + m.group(1)) if m else full[:60]

src, dst = sys.argv[1], sys.argv[2]
out = {}
for leg in ("map-only", "c5-only"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(src, leg, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(src, leg, "kt", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    per = {}
    for k, cs in acc.items():
        if not (k.startswith("k_fuse") or k.startswith("k_smap") or k.startswith("rocprim:")):
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        # reads by request size (TCC_EA0_RDREQ_{128B,64B,32B}): these kernels' scattered 8-B loads are
        # not the wide streaming reads the 2 x FETCH_SIZE correction is calibrated on; 2 x FETCH_SIZE is
        # kept beside it
        rd2 = 2.0 * m.get("FETCH_SIZE", 0.0) * 1024
        sized = 128 * m.get("TCC_EA0_RDREQ_128B", 0.0) + 64 * m.get("TCC_EA0_RDREQ_64B", 0.0) + \
            32 * m.get("TCC_EA0_RDREQ_32B", 0.0)
        rd = sized if sized > 0 else rd2
        wr = m.get("WRITE_SIZE", 0.0) * 1024
        us = sum(dur[k]) / len(dur[k]) if dur.get(k) else None
        per[k[:90]] = {"read_bytes": rd, "read_bytes_2x_fetch_size": rd2, "write_bytes": wr, "avg_us": us,
                       "GB/s": (rd + wr) / (us * 1e-6) / 1e9 if us else None}
    line = [l for l in open(os.path.join(src, leg + ".kt.log")) if l.startswith("{")]
    out[leg] = {"kernels": per, "bench": json.loads(line[-1]) if line else None}
json.dump(out, open(dst, "w"), indent=1)
for leg, v in out.items():
    print(leg)
    for k, d in v["kernels"].items():
        print("  %-60s rd %8.1f MB wr %8.1f MB %8s us" % (k[:60], d["read_bytes"] / 1e6, d["write_bytes"] / 1e6,
                                                          "%.1f" % d["avg_us"] if d["avg_us"] else "-"))
